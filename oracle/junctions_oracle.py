"""CPU oracle for waafle_junctions and waafle_qc (TEST INFRASTRUCTURE ONLY).

A restatement of the reference's algorithms, used by tests/ as the checker for the HIP
junction path (waafle_amd/junctions.py + wf_junctions.hip) and for the QC filter
(waafle_amd/qc.py).  Never imported by the product path.  Pinned by the reference-run
fixtures tests/golden/junc_*.junc.json.gz (make_junctions.py).

  read_pairs         utils.iter_sam_hits / SAMHit / cigar_length (utils.py:524-552)
                     + concordant_hits (waafle_junctions.py:252-275)
  junction_rows      main's coverage / hit loop (:428-451), find_hit_loci (:277-286),
                     evaluate_contig (:292-316), the junction writer (:462-480)
  detailed_rows      write_detailed_output (:318-371)
  qc_filter          waafle_qc.main (waafle_qc.py:133-192)
"""
import csv
import re
from collections import Counter

import numpy as np


def cigar_length(cigar):                                   # utils.py:535-539
    counts = [int(c) for c in re.split("[A-Z]+", cigar) if c != ""]
    sigils = [s for s in re.split("[0-9]+", cigar) if s != ""]
    return sum(c for c, s in zip(counts, sigils) if s in "DHMNSX=")


def sam_hits(path):                                        # utils.py:541-552
    with open(path) as fh:
        for row in csv.reader(fh, dialect="excel-tab"):
            if row[0][0] == "@":
                continue
            elif len(row) < 11:
                continue
            elif row[2] != "*":
                start = int(row[3])
                yield row[0], row[2], start, start + cigar_length(row[5]) - 1


def read_pairs(path):                                      # waafle_junctions.py:252-275
    mate1 = mate2 = None
    for hit in sam_hits(path):
        mate1, mate2 = mate2, hit
        if mate1 is None or mate1[0] != mate2[0] or mate1[1] != mate2[1]:
            continue
        yield mate1, mate2


def calc_overlap(a1, a2, b1, b2):                          # utils.py:487-500, normalize=False
    a1, a2 = sorted([a1, a2])
    b1, b2 = sorted([b1, b2])
    if b1 > a2 or a1 > b2:
        return 0
    outleft, inleft, inright, outright = sorted([a1, a2, b1, b2])
    return inright - inleft + 1


class Locus:                                               # utils.py:298-322
    def __init__(self, row):
        self.start, self.end, self.strand = int(row[3]), int(row[4]), row[6]
        self.code = ":".join([str(self.start), str(self.end), self.strand])

    def __len__(self):
        return abs(self.end - self.start) + 1


def contig_loci(path):                                     # utils.py:341-355 + :421-423
    out = {}
    contig, loci = None, []
    with open(path) as fh:
        for row in csv.reader(fh, csv.excel_tab):
            if row[0][0] == "#":
                continue
            if contig is not None and row[0] != contig:
                out[contig] = loci
                loci = []
            contig = row[0]
            loci.append(Locus(row))
    out[contig] = loci
    return out


def contig_lengths(path):                                  # utils.py:109-120
    data = {}
    header = None
    with open(path) as fh:
        for line in fh:
            line = line.strip()
            if line[0] == ">":
                header = line[1:].split()[0]
                data[header] = 0
            else:
                data[header] += len(line)
    return data


def fmt(v):                                                # utils.py:122-143
    if type(v) in (float, np.float32, np.float64):
        v = "{:.4f}".format(v)
    return str(v) if v != "" else "--"


def accumulate(fna, gff, sam, min_overlap_sites):
    """The main loop of waafle_junctions (:414-451): coverage arrays and gene-pair hits."""
    lengths = contig_lengths(fna)
    coverage = {name: np.zeros(n) for name, n in lengths.items()}
    loci = contig_loci(gff)
    hits_by_contig = {}
    for mate1, mate2 in read_pairs(sam):
        contig = mate1[1]
        inner = hits_by_contig.setdefault(contig, Counter())
        coords = [mate1[2], mate1[3], mate2[2], mate2[3]]
        L, R = min(coords) - 1, max(coords) - 1
        coverage[contig][L:R + 1] += 1
        hits = set()
        for locus in loci.get(contig, []):                 # find_hit_loci (:277-286)
            for read in (mate1, mate2):
                if calc_overlap(locus.start, locus.end, read[2], read[3]) >= min_overlap_sites:
                    hits.add(locus.code)
        for code in hits:
            inner[(code, code)] += 1
        for code1 in hits:
            for code2 in hits:
                if code1 != code2:
                    inner[(code1, code2)] += 1
    return lengths, coverage, loci, hits_by_contig


def junction_rows(fna, gff, sam, min_overlap_sites=25):
    lengths, coverage, loci, hits = accumulate(fna, gff, sam, min_overlap_sites)
    rows = ["\t".join(k.upper() for k in ("contig", "gene1", "gene2", "len_gene1", "len_gene2",
                                          "gap", "junction_hits", "coverage_gene1",
                                          "coverage_gene2", "coverage_junction", "ratio"))]
    with np.errstate(invalid="ignore", divide="ignore"):
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", RuntimeWarning)
            for c in sorted(lengths):                       # evaluate_contig (:292-316)
                ls = sorted(loci.get(c, []), key=lambda x: x.start)
                cov = coverage[c]
                gh = hits.get(c, {})
                for i in range(len(ls) - 1):
                    L1, L2 = ls[i], ls[i + 1]
                    gap = L2.start - L1.end - 1
                    cov1 = np.mean(cov[L1.start - 1:L1.end])
                    cov2 = np.mean(cov[L2.start - 1:L2.end])
                    covj = 0.0 if gap <= 0 else np.mean(cov[L1.end - 1:L2.start])
                    ratio = covj / (np.mean([cov1, cov2]) + 1e-6)
                    rows.append("\t".join(fmt(v) for v in (
                        c, L1.code, L2.code, len(L1), len(L2), gap, gh.get((L1.code, L2.code), 0),
                        cov1, cov2, covj, ratio)))
    return rows


def detailed_rows(fna, gff, sam, min_overlap_sites=25):
    """(site_hits rows, gene_hits rows) of write_detailed_output (:318-371)."""
    lengths, coverage, loci, hits = accumulate(fna, gff, sam, min_overlap_sites)
    site = ["CONTIG\tMEAN\tSTDEV\tDEPTHS"]
    for c in sorted(coverage):
        d = coverage[c]
        site.append("\t".join(fmt(v) for v in (c, np.mean(d), np.std(d),
                                                " ".join("{:.0f}".format(k) for k in d))))
    gene = ["CONTIG\tGENE1\tGENE2\tHITS"]
    for c in sorted(hits):
        for code1, code2 in sorted(hits[c]):
            if code2 > code1:
                continue
            gene.append("\t".join(fmt(v) for v in (c, code1, code2, hits[c][(code1, code2)])))
    return site, gene


def qc_filter(lgt_path, junctions_path, min_junction_hits=2, min_junction_ratio=0.5):
    """waafle_qc.main (waafle_qc.py:133-192): (kept rows incl. header, stderr lines)."""
    say = []
    hits, covs = {}, {}
    say.append("Loading junctions report.")
    with open(junctions_path) as fh:
        reader = csv.reader(fh, dialect="excel-tab")
        headers = next(reader)
        for row in reader:
            R = dict(zip(headers, row))
            key = (R["GENE1"], R["GENE2"])
            hits.setdefault(R["CONTIG"], {})[key] = int(R["JUNCTION_HITS"])
            covs.setdefault(R["CONTIG"], {})[key] = float(R["RATIO"])
    total = failed = 0
    with open(lgt_path) as fh:
        reader = csv.reader(fh, dialect="excel-tab")
        headers = next(reader)
        out = ["\t".join(h.upper() for h in headers)]
        for row in reader:
            R = dict(zip(headers, row))
            total += 1
            contig = R["CONTIG_NAME"]
            if contig not in hits or contig not in covs:
                failed += 1
                say.append("Missing junction data for contig: " + contig)
                continue
            loci = R["LOCI"].split("|")
            synteny = R["SYNTENY"]
            qc_pass = True
            for i in range(len(loci) - 1):
                if synteny[i] + synteny[i + 1] not in ["AB", "BA"]:
                    continue
                gpair = (loci[i], loci[i + 1])
                ok = hits[contig].get(gpair, -1) >= min_junction_hits or \
                    covs[contig].get(gpair, -1) >= min_junction_ratio
                qc_pass = qc_pass and ok
            if not qc_pass:
                failed += 1
                say.append("Failed QC: " + contig)
            else:
                out.append("\t".join(R[h] if R[h] != "" else "--" for h in headers))
    say.append("Failure rate: {} of {} ({:.1f}%)".format(failed, total, 100 * failed / float(total)))
    say.append("Finished successfully.")
    return out, say
