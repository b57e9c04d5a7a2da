"""Parse the four waafle_orgscorer inputs into flat CSR arrays (a `HostBatch`).

Restates the reference readers: FASTA lengths (utils.py:109-120), BLAST rows and
their derived values (utils.py:167-241, grouped by consecutive qseqid :255-270),
GFF loci (utils.py:282-355) and the locus filter / contig bookkeeping of
orgscorer.py:348-357, 908-946.  Columns are converted in bulk with numpy; any row
numpy refuses is re-parsed with the reference's own per-field casts so malformed
input fails the same way.

A contig whose BLAST hits appear in several separate runs of the file keeps them all, in
file order, with each hit's run number (`hit_group`): the scorer reproduces the reference's
evaluation per run (regroup.py).  A contig whose GFF loci appear in two runs is rejected
(upstream re-numbers the second run's loci over the first's names, orgscorer.py:348-357).
"""
from __future__ import annotations

import csv
import os
import sys
from collections import OrderedDict
from dataclasses import dataclass, field

import numpy as np

from .taxonomy import TaxonomyTables, read_edges

BLAST_COLS = 15          # utils.py:167-183
GFF_COLS = 9             # utils.py:282-292
STRAND_CODE = {"+": 0, "-": 1}


class InputError(ValueError):
    """Stands in for utils.die() and the reference's uncaught parse exceptions."""


def say(*args):
    print(" ".join(map(str, args)), file=sys.stderr)


@dataclass
class HostBatch:
    contig_names: list
    contig_lengths: np.ndarray
    hit_off: np.ndarray
    hit_qlo: np.ndarray
    hit_qhi: np.ndarray
    hit_taxon: np.ndarray
    hit_strand: np.ndarray
    hit_score: np.ndarray
    hit_scov: np.ndarray
    hit_sysmask: np.ndarray
    loc_off: np.ndarray
    loc_start: np.ndarray
    loc_end: np.ndarray
    loc_strand: np.ndarray
    loc_codes: list = field(default_factory=list)      # per locus "start:end:strand"
    systems: list = field(default_factory=list)        # annotation system names, bit order
    annot_value_ids: np.ndarray = None                 # [n_hits, n_systems] int32, -1 absent
    annot_values: list = field(default_factory=list)   # per system: list of value strings
    hit_row: np.ndarray = None                         # blastout row of each batch hit
    loci_fields: object = None                         # per contig: LOCI field (native ingest)
    hit_group: np.ndarray = None                       # per hit: its run of the contig (ungrouped blastout)

    @property
    def n_contigs(self):
        return len(self.contig_lengths)

    @property
    def n_hits(self):
        return int(self.hit_off[-1])

    @property
    def n_loci(self):
        return int(self.loc_off[-1])

    @property
    def max_hits(self):
        return int(np.max(np.diff(self.hit_off))) if self.n_contigs else 0

    @property
    def max_loci(self):
        return int(np.max(np.diff(self.loc_off))) if self.n_contigs else 0

    def slice(self, c0, c1):
        """Contigs [c0, c1) as a batch with rebased offsets (hit indices shift by hit_off[c0])."""
        h0, h1 = int(self.hit_off[c0]), int(self.hit_off[c1])
        l0, l1 = int(self.loc_off[c0]), int(self.loc_off[c1])
        return HostBatch(
            contig_names=self.contig_names[c0:c1], contig_lengths=self.contig_lengths[c0:c1],
            hit_off=self.hit_off[c0:c1 + 1] - h0, hit_qlo=self.hit_qlo[h0:h1],
            hit_qhi=self.hit_qhi[h0:h1], hit_taxon=self.hit_taxon[h0:h1],
            hit_strand=self.hit_strand[h0:h1], hit_score=self.hit_score[h0:h1],
            hit_scov=self.hit_scov[h0:h1], hit_sysmask=self.hit_sysmask[h0:h1],
            loc_off=self.loc_off[c0:c1 + 1] - l0, loc_start=self.loc_start[l0:l1],
            loc_end=self.loc_end[l0:l1], loc_strand=self.loc_strand[l0:l1],
            loc_codes=self.loc_codes[l0:l1], systems=self.systems,
            annot_value_ids=None if self.annot_value_ids is None else self.annot_value_ids[h0:h1],
            annot_values=self.annot_values,
            hit_row=None if self.hit_row is None else self.hit_row[h0:h1],
            hit_group=None if self.hit_group is None else self.hit_group[h0:h1],
            loci_fields=None if self.loci_fields is None else _ContigSlice(self.loci_fields, c0, c1))


class _ContigSlice:
    """Entries [c0, c1) of a per-contig string table, without copying it."""

    def __init__(self, table, c0, c1):
        self._t, self._a, self._n = table, c0, c1 - c0

    def __len__(self):
        return self._n

    def __getitem__(self, i):
        if i < 0:
            i += self._n
        return self._t[self._a + i]


# ---------------------------------------------------------------------------
# FASTA (utils.py:109-120)
# ---------------------------------------------------------------------------

def read_contig_lengths(path):
    data = OrderedDict()
    header = None
    with open(path) as fh:
        for line in fh:
            line = line.strip()
            if not line:
                raise InputError("blank line in {} (upstream raises IndexError)".format(path))
            if line[0] == ">":
                parts = line[1:].split()
                if not parts:
                    raise InputError("empty FASTA header in {}".format(path))
                header = parts[0]
                data[header] = 0
            else:
                if header is None:
                    raise InputError("sequence before the first FASTA header in " + path)
                data[header] += len(line)
    return data


# ---------------------------------------------------------------------------
# GFF (utils.py:298-355, orgscorer.py:348-357)
# ---------------------------------------------------------------------------

def read_loci(path, contig_index, min_gene_length, warn=say):
    """Return per-contig lists of kept loci (start, end, strand) in GFF order."""
    per = {}
    seen = set()
    current, group = None, []

    def flush(name, rows):
        if name is None:
            return
        if name not in contig_index:
            if warn:
                warn("  Unknown contig in <gff> file", name)
            return
        if name in seen:
            raise InputError("GFF loci of contig {!r} are not contiguous".format(name))
        seen.add(name)
        kept = [r for r in rows if abs(r[1] - r[0]) + 1 >= min_gene_length]
        per[contig_index[name]] = kept

    with open(path) as fh:
        for row in csv.reader(fh, csv.excel_tab):
            if not row or not row[0]:
                raise InputError("empty GFF row (upstream raises IndexError)")
            if row[0][0] == "#":
                continue
            if len(row) != GFF_COLS:
                raise InputError("Bad GFF row: {}".format(row))
            try:
                start, end = int(row[3]), int(row[4])
                if row[5] != ".":
                    float(row[5])
            except ValueError as exc:
                raise InputError("Bad GFF row: {} ({})".format(row, exc))
            strand = row[6]
            if row[0] != current:
                flush(current, group)
                current, group = row[0], []
            group.append((start, end, strand))
    flush(current, group)
    return per


# ---------------------------------------------------------------------------
# BLAST (utils.py:167-270)
# ---------------------------------------------------------------------------

_INT_COLS = (2, 3, 4, 5, 6, 7, 8, 10, 11)
_FLOAT_COLS = (9, 12, 13)


def _columns(rows):
    cols = list(zip(*rows)) if rows else [()] * BLAST_COLS
    ints = {}
    floats = {}
    try:
        for j in _INT_COLS:
            ints[j] = np.array(cols[j], dtype=np.int64)
        for j in _FLOAT_COLS:
            floats[j] = np.array(cols[j], dtype=np.float64)
    except (ValueError, OverflowError):
        # reproduce the reference's per-row casts (and their exceptions)
        for j in _INT_COLS:
            ints[j] = np.array([int(v) for v in cols[j]], dtype=np.int64)
        for j in _FLOAT_COLS:
            floats[j] = np.array([float(v) for v in cols[j]], dtype=np.float64)
    return cols, ints, floats


def read_hits(path, contig_index, warn=say):
    """Parse the blastout; returns (columns, the runs of known contigs in file order:
    (contig index, row start, row end) -- a contig may have several, utils.py:255-270)."""
    with open(path) as fh:
        rows = list(csv.reader(fh, dialect="excel-tab"))
    for r in rows:
        if len(r) != BLAST_COLS:
            raise InputError("inconsistent blast row: {}".format(r))
    cols, ints, floats = _columns(rows)
    qseqid = cols[0]
    groups = []                       # (contig index, row start, row end)
    start = 0
    n = len(rows)
    for i in range(1, n + 1):
        if i == n or qseqid[i] != qseqid[start]:
            name = qseqid[start]
            if name in contig_index:
                groups.append((contig_index[name], start, i))
            elif warn:
                warn("  Unknown contig in <blastout> file", name)
            start = i
    return rows, cols, ints, floats, groups


def derive_hit_values(qlen, slen, qstart, qend, sstart, send, pident, minus):
    """scov_modified and waafle_score exactly as utils.py:216-229 (same float64 ops)."""
    if np.any(slen == 0) or np.any(qlen == 0):
        raise InputError("float division by zero (slen or qlen is 0 in a BLAST row)")
    s0 = np.where(minus, slen - sstart + 1, sstart)
    s1 = np.where(minus, slen - send + 1, send)
    ltrim = np.maximum(0, s0 - qstart)
    rtrim = np.maximum(0, slen - s0 - qlen + qstart)
    denom = slen - ltrim - rtrim
    if np.any(denom == 0):
        raise InputError("float division by zero (scov_modified denominator is 0)")
    scov = (s1 - s0 + 1) / denom.astype(np.float64)
    score = scov * pident / 100.0
    return scov, score


def split_sseqids(sseqids):
    """taxon = field 1, annotations = 'system=value' fields 2+ (utils.py:231-241)."""
    taxa = []
    annots = []
    for sid in sseqids:
        items = sid.split("|")
        if len(items) < 2:
            raise InputError("bad subject id header: {}".format(sid))
        taxa.append(items[1])
        if len(items) > 2:
            d = {}
            for k in items[2:]:
                parts = k.split("=")
                if len(parts) != 2:
                    raise InputError("bad annotation {!r} in {} (upstream raises "
                                     "ValueError)".format(k, sid))
                d[parts[0]] = parts[1]
            annots.append(d)
        else:
            annots.append(None)
    return taxa, annots


# ---------------------------------------------------------------------------
# assembly
# ---------------------------------------------------------------------------

def load_inputs(contigs_path, blastout_path, gff_path, taxonomy_path, min_gene_length,
                warn=say, native=None, threads=0):
    """Parse all inputs -> (HostBatch, TaxonomyTables).

    native (default: on unless WF_INGEST=python): parse with libwaafle_ingest.so
    (multi-threaded C++); inputs it does not take in its plain form go to the Python
    reader below, which gives the reference's result or error."""
    edges = read_edges(taxonomy_path)
    if native is None:
        native = os.environ.get("WF_INGEST", "native") != "python"
    if native:
        from . import ingest
        try:
            return ingest.parse(contigs_path, blastout_path, gff_path, edges, min_gene_length,
                                threads=threads, warn=warn)
        except ingest.Fallback:
            pass
    return _load_python(contigs_path, blastout_path, gff_path, edges, min_gene_length, warn)


def _load_python(contigs_path, blastout_path, gff_path, edges, min_gene_length, warn):
    lengths = read_contig_lengths(contigs_path)
    names = list(lengths)
    index = {n: i for i, n in enumerate(names)}
    loci = read_loci(gff_path, index, min_gene_length, warn=warn)
    rows, cols, ints, floats, groups = read_hits(blastout_path, index, warn=warn)
    N = len(names)

    # hits reordered into FASTA contig order (file order within a contig, a contig's runs
    # one after another with their run numbers)
    counts = np.zeros(N, dtype=np.int64)
    for ci, a, b in groups:
        counts[ci] += b - a
    hit_off = np.zeros(N + 1, dtype=np.int64)
    np.cumsum(counts, out=hit_off[1:])
    order = np.empty(int(hit_off[-1]), dtype=np.int64)
    run_of = np.zeros(int(hit_off[-1]), dtype=np.int32)
    fill = hit_off[:-1].copy()
    nrun = np.zeros(N, dtype=np.int32)
    for ci, a, b in groups:
        order[fill[ci]:fill[ci] + b - a] = np.arange(a, b)
        run_of[fill[ci]:fill[ci] + b - a] = nrun[ci]
        fill[ci] += b - a
        nrun[ci] += 1

    qlen, slen = ints[2][order], ints[3][order]
    qstart, qend = ints[5][order], ints[6][order]
    sstart, send = ints[7][order], ints[8][order]
    pident = floats[9][order]
    sstrand = [cols[14][i] for i in order.tolist()]
    minus = np.array([s == "minus" for s in sstrand], dtype=bool)
    scov, score = derive_hit_values(qlen, slen, qstart, qend, sstart, send, pident, minus)
    taxa, annots = split_sseqids([cols[1][i] for i in order.tolist()])

    tax = TaxonomyTables(edges, extra_names=set(taxa))
    hit_taxon = np.array([tax.index[t] for t in taxa], dtype=np.int32)

    systems = sorted({s for d in annots if d for s in d})
    if len(systems) > 32:
        raise InputError("more than 32 annotation systems")
    sys_bit = {s: b for b, s in enumerate(systems)}
    sysmask = np.zeros(len(annots), dtype=np.uint32)
    value_ids = np.full((len(annots), max(1, len(systems))), -1, dtype=np.int32)
    values = [[] for _ in systems]
    value_index = [dict() for _ in systems]
    for i, d in enumerate(annots):
        if not d:
            continue
        m = 0
        for s, v in d.items():
            b = sys_bit[s]
            m |= 1 << b
            vi = value_index[b].get(v)
            if vi is None:
                vi = value_index[b][v] = len(values[b])
                values[b].append(v)
            value_ids[i, b] = vi
        sysmask[i] = m

    loc_counts = np.array([len(loci.get(c, ())) for c in range(N)], dtype=np.int64)
    loc_off = np.zeros(N + 1, dtype=np.int64)
    np.cumsum(loc_counts, out=loc_off[1:])
    flat = [r for c in range(N) for r in loci.get(c, ())]
    loc_start = np.array([r[0] for r in flat], dtype=np.int64)
    loc_end = np.array([r[1] for r in flat], dtype=np.int64)
    loc_strand = np.array([STRAND_CODE.get(r[2], 2) for r in flat], dtype=np.int8)
    loc_codes = ["{}:{}:{}".format(r[0], r[1], r[2]) for r in flat]

    for arr, what in ((qstart, "qstart"), (qend, "qend"), (loc_start, "gff start"),
                      (loc_end, "gff end")):
        if len(arr) and (arr.min() < -(2 ** 31) or arr.max() >= 2 ** 31):
            raise InputError("{} outside int32".format(what))

    batch = HostBatch(
        contig_names=names, contig_lengths=np.array([lengths[n] for n in names], dtype=np.int64),
        hit_off=hit_off, hit_qlo=np.minimum(qstart, qend).astype(np.int32),
        hit_qhi=np.maximum(qstart, qend).astype(np.int32), hit_taxon=hit_taxon,
        hit_strand=minus.astype(np.int8), hit_score=score.astype(np.float64),
        hit_scov=scov.astype(np.float64), hit_sysmask=sysmask, loc_off=loc_off,
        loc_start=loc_start.astype(np.int32), loc_end=loc_end.astype(np.int32),
        loc_strand=loc_strand, loc_codes=loc_codes, systems=systems,
        annot_value_ids=value_ids, annot_values=values, hit_row=order,
        hit_group=run_of if np.any(run_of) else None)
    return batch, tax


def basename_of(contigs_path):
    """orgscorer.py:928-929."""
    return os.path.split(contigs_path)[1].split(".")[0]
