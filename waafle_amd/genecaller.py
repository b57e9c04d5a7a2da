"""`waafle_genecaller` on the GPU: gene calls (GFF) from a blastout.

    python -m waafle_amd.genecaller <blastout> [--gff PATH] [--min-overlap 0.1]
                                    [--min-gene-length 200] [--min-scov 0.75] [--stranded]

Same arguments, defaults and output as the reference (waafle_genecaller.py:44-101, main
:199-237).  The blastout is read in file order and grouped by consecutive qseqid
(utils.py:255-270); every group's intervals are clustered and merged by the HIP kernel
behind `wf_genecall` (waafle_amd/csrc/wf_genecall.hip).  There is no CPU fallback.
As upstream, --stranded has no effect: the reference tests `args.stranded == "on"` on a
store_true flag (waafle_genecaller.py:212-215).
"""
import argparse
import csv
import ctypes as C
import os
import sys

import numpy as np

from . import lib as L
from .inputs import BLAST_COLS, InputError, _columns, derive_hit_values


class GeneCalls:
    """Per contig group (blastout order): name and (start, stop, strand char) genes."""

    def __init__(self, names, genes):
        self.names = names
        self.genes = genes

    def rows(self):
        out = []
        for name, gl in zip(self.names, self.genes):
            for start, stop, strand in gl:
                out.append([name, "waafle_genecaller", "gene", str(start), str(stop), ".",
                            strand, "0", "."])
        return out


def read_groups(path):
    """Blastout -> (group names, hit_off, qstart, qend, strand 0/1, scov) in file order."""
    with open(path) as fh:
        rows = list(csv.reader(fh, dialect="excel-tab"))
    for r in rows:
        if len(r) != BLAST_COLS:
            raise InputError("inconsistent blast row: {}".format(r))
    cols, ints, floats = _columns(rows)
    n = len(rows)
    names, off = [], [0]
    for i in range(1, n + 1):
        if i == n or cols[0][i] != cols[0][off[-1]]:
            names.append(cols[0][off[-1]])
            off.append(i)
    if n == 0:
        off = [0]
    minus = np.array([s == "minus" for s in cols[14]], dtype=bool) if n else np.zeros(0, bool)
    if n:
        scov, _ = derive_hit_values(ints[2], ints[3], ints[5], ints[6], ints[7], ints[8],
                                    floats[9], minus)
    else:
        scov = np.zeros(0)
    return (names, np.array(off, dtype=np.int64), ints[5].astype(np.int32) if n else np.zeros(0, np.int32),
            ints[6].astype(np.int32) if n else np.zeros(0, np.int32), minus.astype(np.int8),
            np.ascontiguousarray(scov, dtype=np.float64))


def call_genes(path, min_overlap=0.1, min_gene_length=200.0, min_scov=0.75, device=0):
    names, off, qs, qe, strand, scov = read_groups(path)
    G, NH = len(names), int(off[-1])
    n_genes = np.zeros(max(G, 1), dtype=np.int32)
    gs = np.zeros(max(NH, 1), dtype=np.int32)
    ge = np.zeros(max(NH, 1), dtype=np.int32)
    gst = np.zeros(max(NH, 1), dtype=np.int8)
    so = L.load()
    h = C.c_void_p()
    rc = so.wf_init(device, C.byref(h))
    if rc:
        raise L.WaafleHipError(rc, "wf_init failed")
    try:
        b = L.WfGcBatch(n_groups=G, device_resident=0, n_hits=NH, hit_off=L.ptr(off),
                        hit_qlo=L.ptr(qs), hit_qhi=L.ptr(qe), hit_strand=L.ptr(strand),
                        hit_scov=L.ptr(scov))
        p = L.WfGcParams(min_overlap=min_overlap, min_scov=min_scov,
                         min_gene_length=min_gene_length, stranded=0)
        r = L.WfGcResult(n_genes=L.ptr(n_genes), gene_start=L.ptr(gs), gene_stop=L.ptr(ge),
                         gene_strand=L.ptr(gst))
        rc = so.wf_genecall(h, C.byref(b), C.byref(p), C.byref(r))
        if rc:
            raise L.WaafleHipError(rc, so.wf_last_error(h).decode())
    finally:
        so.wf_free(h)
    genes = []
    for g in range(G):
        o = int(off[g])
        k = int(n_genes[g])
        genes.append([(int(gs[o + i]), int(ge[o + i]), "-" if gst[o + i] else "+")
                      for i in range(k)])
    return GeneCalls(names, genes)


def write_gff(calls, path):
    with open(path, "w", newline="") as fh:
        w = csv.writer(fh, csv.excel_tab)
        for row in calls.rows():
            w.writerow(row)


def get_args(argv=None):
    ap = argparse.ArgumentParser(
        description="waafle_genecaller on MI355X: gene calls from a waafle_search blastout")
    ap.add_argument("blastout", help="(custom) blast output from waafle_search")
    ap.add_argument("--gff", default=None, metavar="<path>",
                    help="path for (output) waafle gene calls (.gff) [default: <derived from input>]")
    ap.add_argument("--min-overlap", default=0.1, type=float, metavar="<float>")
    ap.add_argument("--min-gene-length", default=200, type=float, metavar="<int>")
    ap.add_argument("--min-scov", default=0.75, type=float, metavar="<float>")
    ap.add_argument("--stranded", action="store_true",
                    help="accepted; no effect (as upstream)")
    return ap.parse_args(argv)


def main(argv=None):
    args = get_args(argv)
    if args.gff is None:                              # utils.py path2name / name2path
        name = os.path.split(args.blastout)[1].split(".")[0]
        args.gff = os.path.join(".", name + ".gff")
    calls = call_genes(args.blastout, args.min_overlap, args.min_gene_length, args.min_scov)
    write_gff(calls, args.gff)
    print("Finished successfully.", file=sys.stderr)


if __name__ == "__main__":
    main()
