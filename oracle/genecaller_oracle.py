"""ORACLE -- TEST INFRASTRUCTURE, NOT PRODUCT CODE.

CPU restatement of the reference `waafle_genecaller` (menickname/waafle v0.1.0,
waafle/waafle_genecaller.py) used only by `tests/` to check the HIP path behind
`wf_genecall`.  Pinned by the reference's own shipped golden: demo/output/demo_contigs.gff
is waafle_genecaller's output on demo/output/demo_contigs.blastout with default flags
(copied as tests/golden/demo_inputs/demo_contigs.{blastout,gff}.gz; see
tests/test_genecaller.py).

It follows the reference step by step, including its O(n^2) pair scan with the early
`break` and its breadth-first connected components, so it is an independent check of the
kernel's sort + hooking formulation.
"""
from .orgscorer_oracle import blast_groups


def calc_overlap(a1, a2, b1, b2):
    """utils.py:487-500 (normalize=True)."""
    a1, a2 = sorted([a1, a2])
    b1, b2 = sorted([b1, b2])
    if b1 > a2 or a1 > b2:
        return 0
    _, inleft, inright, _ = sorted([a1, a2, b1, b2])
    return (inright - inleft + 1) / float(min(a2 - a1 + 1, b2 - b1 + 1))


class INode:
    """utils.py:455-485 (interval node)."""

    def __init__(self, start, stop, strand="+"):
        self.start, self.stop = sorted([start, stop])
        self.strand = strand
        self.neighbors = []
        self.visited = False

    def __len__(self):
        return self.stop - self.start + 1

    def component(self):
        """get_connected_component :471-482: every inode reachable from this one (the
        merge below only depends on membership)."""
        cc, stack = [], [self]
        self.visited = True
        while stack:
            n = stack.pop()
            cc.append(n)
            for m in n.neighbors:
                if not m.visited:
                    m.visited = True
                    stack.append(m)
        return cc


def overlap_intervals(intervals, threshold, stranded=False):
    """waafle_genecaller.py:138-170."""
    inodes = [INode(a, b, s) for a, b, s in intervals]
    inodes = sorted(inodes, key=lambda n: n.start)                  # stable
    for i, n1 in enumerate(inodes):
        for n2 in inodes[i + 1:]:
            if not stranded or n1.strand == n2.strand:
                score = calc_overlap(n1.start, n1.stop, n2.start, n2.stop)
                if score >= threshold:
                    n1.neighbors.append(n2)
                    n2.neighbors.append(n1)
                elif score == 0:
                    break
    out = []
    for n in inodes:
        if not n.visited:
            cc = n.component()
            start = min(m.start for m in cc)                           # merge_inodes :125-136
            stop = max(m.stop for m in cc)
            strand = sorted([len(m), m.strand] for m in cc)[-1][1]
            out.append((start, stop, strand))
    return out


def call_genes(blastout, min_overlap=0.1, min_gene_length=200.0, min_scov=0.75,
               stranded=False):
    """main loop :199-233: [(contig, [(start, stop, strand), ...]), ...] in file order."""
    res = []
    for contig, hits in blast_groups(blastout):
        if contig is None:
            continue
        ints = [(h.qstart, h.qend, h.strand) for h in hits if h.scov_mod >= min_scov]
        genes = [g for g in overlap_intervals(ints, min_overlap, stranded)
                 if g[1] - g[0] + 1 >= min_gene_length]
        res.append((contig, genes))
    return res


def gff_rows(calls):
    rows = []
    for contig, genes in calls:
        for start, stop, strand in genes:
            rows.append([contig, "waafle_genecaller", "gene", str(start), str(stop), ".",
                         strand, "0", "."])
    return rows
