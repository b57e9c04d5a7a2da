"""`waafle_junctions` drop-in (waafle_junctions.py) with the per-pair work on MI355X.

    python -m waafle_amd.junctions contigs.fna genes.gff --sam reads.sam [options]

Host side (this module): the reference's readers -- FASTA lengths (utils.py:109-120), GFF
loci grouped by contig (utils.py:298-355; a contig's last group wins, as the reference's
dict assignment at :421-423), SAM records (utils.py:524-552) paired by the reference's
sliding window (concordant_hits, waafle_junctions.py:252-275) -- and the writers
(:318-371, :462-480).  Device side (wf_junctions, wf_junctions.hip): per-site coverage of
every concordant pair, the pair's hit loci and the junction table (evaluate_contig,
:292-316).  bowtie2 is only run when reads are given (as upstream, :196-246).
"""
from __future__ import annotations

import argparse
import ctypes as C
import csv
import gzip
import os
import re
import sys
from collections import Counter

import numpy as np

from . import inputs, lib as L

JUNCTION_FIELDS = ["contig", "gene1", "gene2", "len_gene1", "len_gene2", "gap", "junction_hits",
                   "coverage_gene1", "coverage_gene2", "coverage_junction", "ratio"]
SITE_FIELDS = ["contig", "mean", "stdev", "depths"]
GENE_FIELDS = ["contig", "gene1", "gene2", "hits"]


class JunctionError(RuntimeError):
    pass


def die(*args):
    inputs.say(*(["LETHAL ERROR:"] + list(args)))
    sys.exit("EXITING.")


# ---------------------------------------------------------------------------
# readers
# ---------------------------------------------------------------------------

class GffLocus:
    """utils.Locus (utils.py:298-322): start/end ints, code "start:end:strand"."""
    __slots__ = ("start", "end", "strand", "code")

    def __init__(self, row):
        if len(row) != 9:
            raise JunctionError("Bad GFF row: {}".format(row))
        start = int(row[3]) if row[3] != "." else "."
        end = int(row[4]) if row[4] != "." else "."
        if row[5] != ".":
            float(row[5])
        if start == "." or end == ".":
            raise JunctionError("GFF row without coordinates: {}".format(row))
        self.start, self.end, self.strand = start, end, row[6]
        self.code = "{}:{}:{}".format(start, end, row[6])

    def __len__(self):
        return abs(self.end - self.start) + 1


def read_contig_loci(path):
    """{contig: [GffLocus]} as iter_contig_loci + the dict of waafle_junctions.py:421-423."""
    out = {}
    contig, loci = None, []
    with open(path) as fh:
        for row in csv.reader(fh, csv.excel_tab):
            if not row or not row[0]:
                raise JunctionError("empty GFF row (upstream raises IndexError)")
            if row[0][0] == "#":
                continue
            locus = GffLocus(row)
            if contig is not None and row[0] != contig:
                out[contig] = loci
                loci = []
            contig = row[0]
            loci.append(locus)
    out[contig] = loci
    out.pop(None, None)
    return out


_STD_CIGAR = re.compile(r"^(?:[0-9]+[MIDNSHPX])+$")
_CIGAR_OP = re.compile(r"([0-9]+)([MIDNSHPX])")


def cigar_length(cigar):
    """utils.cigar_length (utils.py:535-539): sum of the D, H, M, N, S, X counts."""
    if _STD_CIGAR.match(cigar):
        return sum(int(n) for n, op in _CIGAR_OP.findall(cigar) if op in "DHMNSX")
    counts = [int(c) for c in re.split("[A-Z]+", cigar) if c != ""]      # raises as upstream
    sigils = [s for s in re.split("[0-9]+", cigar) if s != ""]
    return sum(c for c, s in zip(counts, sigils) if s in "DHMNSX=")


def read_pairs(path, contig_index):
    """Concordant pairs of the SAM file (utils.iter_sam_hits + concordant_hits): arrays
    (pair_contig, m1_start, m1_end, m2_start, m2_end) plus the contig names of the pairs
    whose contig is not in the FASTA (the reference fails on those with a KeyError)."""
    pc, m1s, m1e, m2s, m2e = [], [], [], [], []
    missing = []
    prev = None
    with open(path) as fh:
        for row in csv.reader(fh, dialect="excel-tab"):
            if row[0][0] == "@":                  # IndexError on an empty row, as upstream
                continue
            if len(row) < 11 or row[2] == "*":
                continue
            start = int(row[3])
            hit = (row[0], row[2], start, start + cigar_length(row[5]) - 1)
            if prev is not None and prev[0] == hit[0] and prev[1] == hit[1]:
                c = contig_index.get(hit[1])
                if c is None:
                    missing.append(hit[1])
                else:
                    pc.append(c)
                    m1s.append(prev[2]); m1e.append(prev[3])
                    m2s.append(hit[2]); m2e.append(hit[3])
            prev = hit
    as64 = lambda v: np.array(v, dtype=np.int64)
    return np.array(pc, dtype=np.int32), as64(m1s), as64(m1e), as64(m2s), as64(m2e), missing


# ---------------------------------------------------------------------------
# device call
# ---------------------------------------------------------------------------

class JunctionTable:
    """Host arrays of one wf_junctions call (loci in per-contig start order)."""

    def __init__(self, names, lengths, loci_by_contig):
        self.names = list(names)
        self.lengths = np.asarray(lengths, dtype=np.int64)
        self.loci = []
        off = [0]
        for n in self.names:
            ls = sorted(loci_by_contig.get(n, []), key=lambda x: x.start)   # stable, :296
            self.loci.extend(ls)
            off.append(len(self.loci))
        self.loc_off = np.array(off, dtype=np.int64)
        self.loc_start = np.array([l.start for l in self.loci], dtype=np.int64)
        self.loc_end = np.array([l.end for l in self.loci], dtype=np.int64)


def score_junctions(table, pairs, min_overlap_sites=25, device=0, coverage=False,
                    locus_hits=False, pair_sets=False):
    """Run wf_junctions; returns a dict of result arrays (per locus j: the junction j, j+1)."""
    so = L.load()
    h = C.c_void_p()
    rc = so.wf_init(int(device), C.byref(h))
    if rc != L.WF_OK:
        raise L.WaafleHipError(rc, "wf_init(device={}) failed".format(device))
    try:
        pc, m1s, m1e, m2s, m2e = [np.ascontiguousarray(a) for a in pairs[:5]]
        NL = len(table.loci)
        out = dict(junction_hits=np.zeros(NL, np.int32), coverage_gene1=np.zeros(NL),
                   coverage_gene2=np.zeros(NL), coverage_junction=np.zeros(NL),
                   ratio=np.zeros(NL))
        if locus_hits:
            out["locus_hits"] = np.zeros(NL, np.int32)
        if coverage:
            out["coverage"] = np.zeros(int(table.lengths.sum()), np.int64)
        if pair_sets:
            out["pair_first"] = np.zeros(len(pc), np.int64)
            out["pair_mask"] = np.zeros(len(pc), np.uint64)
        b = L.WfJnBatch(n_contigs=len(table.names), device_resident=0, n_pairs=len(pc),
                        n_loci=NL, contig_length=L.ptr(table.lengths), loc_off=L.ptr(table.loc_off),
                        loc_start=L.ptr(table.loc_start), loc_end=L.ptr(table.loc_end),
                        pair_contig=L.ptr(pc), m1_start=L.ptr(m1s), m1_end=L.ptr(m1e),
                        m2_start=L.ptr(m2s), m2_end=L.ptr(m2e))
        p = L.WfJnParams(min_overlap_sites=int(min_overlap_sites))
        r = L.WfJnResult(**{f: L.ptr(out.get(f)) for f, _ in L.WfJnResult._fields_})
        rc = so.wf_junctions(h, C.byref(b), C.byref(p), C.byref(r))
        if rc != L.WF_OK:
            raise L.WaafleHipError(rc, so.wf_last_error(h).decode())
        return out
    finally:
        so.wf_free(h)


# ---------------------------------------------------------------------------
# writers (utils.write_rowdict: uppercase headers, %.4f floats, "" -> "--")
# ---------------------------------------------------------------------------

def _fmt(v):
    if isinstance(v, (float, np.floating)):
        return "{:.4f}".format(float(v))
    s = str(v)
    return s if s != "" else "--"


def _row(values):
    return "\t".join(_fmt(v) for v in values)


def junction_rows(table, res):
    """evaluate_contig rows (waafle_junctions.py:292-316) for contigs in sorted order."""
    lines = ["\t".join(f.upper() for f in JUNCTION_FIELDS)]
    order = sorted(range(len(table.names)), key=lambda c: table.names[c])
    for c in order:
        for j in range(int(table.loc_off[c]), int(table.loc_off[c + 1]) - 1):
            L1, L2 = table.loci[j], table.loci[j + 1]
            lines.append(_row([table.names[c], L1.code, L2.code, len(L1), len(L2),
                               L2.start - L1.end - 1, int(res["junction_hits"][j]),
                               res["coverage_gene1"][j], res["coverage_gene2"][j],
                               res["coverage_junction"][j], res["ratio"][j]]))
    return lines


def site_rows(table, coverage):
    """write_detailed_output site hits (:330-345): every FASTA contig, sorted."""
    lines = ["\t".join(f.upper() for f in SITE_FIELDS)]
    starts = np.concatenate([[0], np.cumsum(table.lengths)])
    for c in sorted(range(len(table.names)), key=lambda c: table.names[c]):
        depths = coverage[starts[c]:starts[c + 1]].astype(np.float64)
        lines.append(_row([table.names[c], np.mean(depths), np.std(depths),
                           " ".join("{:.0f}".format(k) for k in depths)]))
    return lines


def gene_hit_rows(table, pairs, res):
    """write_detailed_output gene-pair hits (:347-371) from the device's per-pair hit sets:
    per contig with >= 1 concordant pair, every stored (code1, code2) key with
    code2 <= code1, sorted.  A pair adds 1 to (x, x) for each code x it hits and to (x, y)
    for each ordered pair of distinct codes (:437-451)."""
    lines = ["\t".join(f.upper() for f in GENE_FIELDS)]
    pc = np.asarray(pairs[0], dtype=np.int64)
    first, mask = res["pair_first"], res["pair_mask"]
    codes = sorted({l.code for l in table.loci})
    code_id = {c: i for i, c in enumerate(codes)}
    loc_code = np.array([code_id[l.code] for l in table.loci], dtype=np.int64)
    # (pair, code) hits, one per distinct code of a pair
    pp, cc = [], []
    for bit in range(64):
        sel = (first >= 0) & (((mask >> np.uint64(bit)) & np.uint64(1)) == 1)
        idx = np.nonzero(sel)[0]
        pp.append(idx)
        cc.append(loc_code[first[idx] + bit])
    P = np.concatenate(pp).astype(np.int64)
    K = np.concatenate(cc).astype(np.int64)
    ncode = max(len(codes), 1)
    u = np.unique(P * ncode + K)
    P, K = u // ncode, u % ncode
    # all ordered (x, y) of each pair's set, x == y included (the self counts)
    starts = np.searchsorted(P, np.unique(P)).astype(np.int64)
    sizes = np.diff(np.concatenate([starts, [len(P)]])).astype(np.int64)
    sq = sizes * sizes
    T = int(sq.sum())
    grp = np.repeat(np.arange(len(sizes)), sq)
    local = np.arange(T) - np.repeat(np.cumsum(sq) - sq, sq)
    sz = np.maximum(sizes[grp], 1)
    xa = K[starts[grp] + local // sz]
    xb = K[starts[grp] + local % sz]
    contig = pc[P[starts[grp]]]
    key = (contig * ncode + xa) * ncode + xb
    ukey, cnt = np.unique(key, return_counts=True)
    per = {}
    for k, n in zip(ukey.tolist(), cnt.tolist()):
        c, rest = divmod(k, ncode * ncode)
        a, b2 = divmod(rest, ncode)
        per.setdefault(table.names[c], []).append((codes[a], codes[b2], n))
    # contigs with a concordant pair but no hit keep an empty Counter: no rows
    for name in sorted(per):
        for code1, code2, n in sorted(per[name]):
            if code2 > code1:
                continue
            lines.append(_row([name, code1, code2, n]))
    return lines


# ---------------------------------------------------------------------------
# CLI (waafle_junctions.py:96-190, 374-483)
# ---------------------------------------------------------------------------

def build_parser():
    ap = argparse.ArgumentParser(description="waafle_junctions on MI355X: gene-gene junction "
                                             "stats for contig QC",
                                 formatter_class=argparse.RawTextHelpFormatter)
    g = ap.add_argument_group("required inputs")
    g.add_argument("contigs", help="contigs file (fasta format)")
    g.add_argument("gff", help="GFF file for provided contigs")
    g = ap.add_argument_group("provide paired reads or a .sam file")
    g.add_argument("--reads1", metavar="<path>", help="sequencing reads (mate-1)")
    g.add_argument("--reads2", metavar="<path>", help="sequencing reads (mate-2)")
    g.add_argument("--sam", metavar="<path>", help="sam file (from existing alignment)")
    g = ap.add_argument_group("output options")
    g.add_argument("--tmpdir", default=".", metavar="<path>",
                   help="where to place temp outputs\n[default: ./]")
    g.add_argument("--outdir", default=".", metavar="<path>",
                   help="where to place main outputs\n[default: ./]")
    g.add_argument("--basename", metavar="<str>",
                   help="basename for output files\n[default: <derived from input>]")
    g.add_argument("--write-detailed-output", action="store_true",
                   help="write out coverage values for all sites and all junctions\n[default: off]")
    g = ap.add_argument_group("filtering parameters")
    g.add_argument("--min-overlap-sites", type=int, default=25, metavar="<int>",
                   help="minimum nucleotide overlap for counting a read-gene hit\n[default: 25]")
    g = ap.add_argument_group("bowtie2 options")
    g.add_argument("--bowtie2-build", default="bowtie2-build", metavar="<path>",
                   help="path to bowtie2-build\n[default: $PATH]")
    g.add_argument("--bowtie2", default="bowtie2", metavar="<path>",
                   help="path to bowtie2\n[default: $PATH]")
    g.add_argument("--threads", type=int, default=1, metavar="<int>",
                   help="number of threads for bowtie2 steps\n[default: 1]")
    g.add_argument("--resume", action="store_true",
                   help="if set, use existing .index and/or .sam if found\n[default: off]")
    g.add_argument("--gpu", type=int, default=0, help="device to run on (MI355X build)")
    return ap


def _bowtie2(args, p_index, p_sam):
    """bowtie2_build + bowtie2_align (waafle_junctions.py:196-246), same commands."""
    import subprocess
    if not (args.resume and os.path.exists(p_index + ".1.bt2")):
        inputs.say("Indexing <{}> to <{}>.".format(args.contigs, p_index))
        subprocess.run("{} {} {}".format(args.bowtie2_build, args.contigs, p_index), shell=True)
    if not (args.resume and os.path.exists(p_sam)):
        inputs.say("Performing bowtie2 alignment.")
        subprocess.run("{} -x {} -1 {} -2 {} -S {} --threads {} --no-mixed --no-discordant".format(
            args.bowtie2, p_index, args.reads1, args.reads2, p_sam, args.threads), shell=True)


def main(argv=None):
    args = build_parser().parse_args(argv)
    basename = args.basename or inputs.basename_of(args.contigs)
    p_sam = os.path.join(args.tmpdir, basename + ".sam")
    if args.sam is not None:
        p_sam = args.sam
        inputs.say("Using specified SAM file:", p_sam)
    elif args.reads1 is not None and args.reads2 is not None:
        _bowtie2(args, os.path.join(args.tmpdir, basename + ".index"), p_sam)
    else:
        die("Must provide READS or SAM file.")
    try:
        lengths = inputs.read_contig_lengths(args.contigs)
        loci = read_contig_loci(args.gff)
        names = list(lengths)
        pairs = read_pairs(p_sam, {n: i for i, n in enumerate(names)})
    except (inputs.InputError, JunctionError, ValueError) as exc:
        die(str(exc))
    if pairs[5]:
        die("SAM alignment to a contig missing from the FASTA:", pairs[5][0])
    table = JunctionTable(names, [lengths[n] for n in names], loci)
    try:
        res = score_junctions(table, pairs, args.min_overlap_sites, device=args.gpu,
                              coverage=args.write_detailed_output,
                              pair_sets=args.write_detailed_output)
    except L.WaafleHipError as exc:
        die(str(exc))
    if args.write_detailed_output:
        with gzip.open(os.path.join(args.outdir, basename + ".site_hits.tsv.gz"), "wt") as fh:
            fh.write("\n".join(site_rows(table, res["coverage"])) + "\n")
        with open(os.path.join(args.outdir, basename + ".gene_hits.tsv"), "w") as fh:
            fh.write("\n".join(gene_hit_rows(table, pairs, res)) + "\n")
    with open(os.path.join(args.outdir, basename + ".junctions.tsv"), "w") as fh:
        fh.write("\n".join(junction_rows(table, res)) + "\n")
    inputs.say("Finished successfully.")


if __name__ == "__main__":
    main()
