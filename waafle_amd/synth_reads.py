"""Seeded synthetic paired-read alignments (SAM) over a synthetic contig set.

Input for waafle_junctions / waafle_qc.  bowtie2 is not in this
image, so the mapping step is replaced by alignments drawn directly on the contigs, in
the record shape bowtie2 writes (`--no-mixed --no-discordant`, waafle_junctions.py:
228-246) plus the irregular records a real file carries, so the reference's reader
(utils.py:524-552) and pairing rule (waafle_junctions.py:252-275) see every case:

  * concordant pairs: two consecutive records with the same QNAME and RNAME;
  * singletons, unmapped records (RNAME "*"), pairs split across contigs;
  * a third record for a QNAME (the reference pairs records with a sliding window, so a
    triple yields two pairs);
  * CIGARs with soft/hard clips, insertions, deletions and skips (cigar_length counts
    D, H, M, N, S, X, =), and reads running past the contig end;
  * header lines and short rows (< 11 fields), which the reader skips.
"""
from __future__ import annotations

import numpy as np

CIGARS = ["100M", "100M", "100M", "100M", "20S80M", "50M2I48M", "45M5D55M", "60M300N40M",
          "10H90M", "95M5S", "30M1D20M1I49M", "50M2X48M"]


def sam_records(data, pairs_per_kb=3.0, seed=0, insert=(150, 600), skip_frac=0.05):
    """SAM lines (header + records) for SynthData `data`."""
    rng = np.random.default_rng(seed)
    names = data.contig_names
    lengths = data.contig_lengths.tolist()
    out = ["@HD\tVN:1.0\tSO:unsorted"]
    out += ["@SQ\tSN:{}\tLN:{}".format(n, l) for n, l in zip(names, lengths)]
    out.append("short\trow")                                     # < 11 fields: skipped
    q = 0

    def rec(qname, flag, rname, pos, cigar):
        return "\t".join([qname, str(flag), rname, str(pos), "42", cigar, "=", "0", "0",
                          "N", "I"])

    for ci, (name, L) in enumerate(zip(names, lengths)):
        if rng.random() < skip_frac:
            continue                                             # contig without reads
        n = rng.poisson(max(1.0, pairs_per_kb * L / 1000.0))
        for _ in range(int(n)):
            q += 1
            qname = "read{}".format(q)
            ins = int(rng.integers(insert[0], insert[1]))
            p1 = int(rng.integers(1, max(2, L - 50)))            # may run past the end
            p2 = max(1, p1 + ins - 100)
            c1, c2 = CIGARS[rng.integers(len(CIGARS))], CIGARS[rng.integers(len(CIGARS))]
            kind = rng.random()
            first = [rec(qname, 99, name, p1, c1)]
            second = [rec(qname, 147, name, p2, c2)]
            if kind < 0.03:                                      # singleton
                second = []
            elif kind < 0.05:                                    # mate on another contig
                other = names[(ci + 1 + int(rng.integers(len(names) - 1))) % len(names)] \
                    if len(names) > 1 else name
                second = [rec(qname, 147, other, p2, c2)]
            elif kind < 0.07:                                    # unmapped mate
                second = [rec(qname, 141, "*", 0, "*")]
            elif kind < 0.08:                                    # a third record
                second.append(rec(qname, 2048 + 147, name, max(1, p2 - 37), "100M"))
            if rng.random() < 0.5:
                first, second = second, first
            out += first + second
    for k in range(3):                                           # fully unmapped pairs
        out.append(rec("unmapped{}".format(k), 77, "*", 0, "*"))
        out.append(rec("unmapped{}".format(k), 141, "*", 0, "*"))
    return out


def write_sam(data, path, **kw):
    with open(path, "w") as fh:
        fh.write("\n".join(sam_records(data, **kw)) + "\n")
    return path
