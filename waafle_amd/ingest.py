"""ctypes binding of libwaafle_ingest.so (include/waafle_ingest.h): native multi-threaded
parsing of the FASTA / BLAST / GFF inputs into a `HostBatch`.

The native parser takes the plain spelling of every field; for anything else (including
every malformed input) it reports a fallback and `load_inputs` runs the Python reader
(`inputs.py`), which accepts the unusual spelling or raises the reference's error.  The
two readers produce identical batches (tests/test_ingest.py).
"""
import ctypes as C
import os

import numpy as np

from .taxonomy import TaxonomyTables

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libwaafle_ingest.so")

INGEST_OK, INGEST_FALLBACK, INGEST_E_IO, INGEST_E_STATE = 0, 1, -1, -2

_P = C.c_void_p


class WfIngestView(C.Structure):
    _fields_ = [("n_contigs", C.c_int32), ("n_taxa", C.c_int32), ("n_systems", C.c_int32),
                ("n_warn_gff", C.c_int32), ("n_warn_blast", C.c_int32), ("_pad", C.c_int32),
                ("n_hits", C.c_int64), ("n_loci", C.c_int64), ("n_values", C.c_int64),
                ("contig_blob", _P), ("contig_off", _P), ("contig_length", _P),
                ("hit_off", _P), ("hit_qlo", _P), ("hit_qhi", _P), ("hit_taxon", _P),
                ("hit_strand", _P), ("hit_score", _P), ("hit_scov", _P), ("hit_sysmask", _P),
                ("hit_row", _P), ("hit_value", _P),
                ("taxa_blob", _P), ("taxa_off", _P), ("system_blob", _P), ("system_off", _P),
                ("value_blob", _P), ("value_off", _P), ("value_system", _P),
                ("loc_off", _P), ("loc_start", _P), ("loc_end", _P), ("loc_strand", _P),
                ("loc_strand_blob", _P), ("loc_strand_off", _P),
                ("warn_gff_blob", _P), ("warn_gff_off", _P),
                ("warn_blast_blob", _P), ("warn_blast_off", _P),
                ("loci_blob", _P), ("loci_off", _P), ("hit_group", _P)]


class IngestError(RuntimeError):
    pass


class Fallback(Exception):
    """The input needs the Python reader (message says why)."""


_lib = None


def load(path=LIB_PATH):
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise IngestError("{} is missing: build it with `python -m waafle_amd.build`".format(path))
    so = C.CDLL(path)
    so.wf_ingest_abi_version.restype = C.c_int
    so.wf_ingest_new.restype = _P
    so.wf_ingest_free.argtypes = [_P]
    so.wf_ingest_last_error.argtypes = [_P]
    so.wf_ingest_last_error.restype = C.c_char_p
    so.wf_ingest_parse.argtypes = [_P, C.c_char_p, C.c_char_p, C.c_char_p, C.c_double, C.c_int]
    so.wf_ingest_parse.restype = C.c_int
    so.wf_ingest_get_view.argtypes = [_P, C.POINTER(WfIngestView)]
    so.wf_ingest_get_view.restype = C.c_int
    if so.wf_ingest_abi_version() != 3:
        raise IngestError("libwaafle_ingest.so ABI mismatch")
    _lib = so
    return so


class _Owner:
    """Keeps a parsed wf_ingest object (and the arrays it owns) alive; the numpy arrays
    handed out are views of its memory and hold a reference to it."""

    def __init__(self, so, h):
        self.so, self.h = so, h

    def __del__(self):
        if self.h:
            self.so.wf_ingest_free(self.h)
            self.h = None


def _arr(ptr, n, dtype, owner=None):
    """n elements at ptr as a numpy array: a view of the native memory kept alive by
    `owner`, or a copy when there is none."""
    if n == 0 or not ptr:
        return np.zeros(0, dtype=dtype)
    buf = (C.c_char * (n * np.dtype(dtype).itemsize)).from_address(ptr)
    if owner is None:
        return np.frombuffer(buf, dtype=dtype, count=n).copy()
    buf._owner = owner
    return np.frombuffer(buf, dtype=dtype, count=n)


class StringTable:
    """Read-only list of strings kept as one ASCII blob + offsets, decoded on access (the
    annotation value table can hold one text per hit)."""

    def __init__(self, blob, off):
        self._blob, self._off = blob, off

    def __len__(self):
        return len(self._off) - 1

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(len(self)))]
        if i < 0:
            i += len(self)
        return bytes(self._blob[self._off[i]:self._off[i + 1]]).decode("ascii")

    def __iter__(self):
        return (self[i] for i in range(len(self)))

    def __eq__(self, other):
        return list(self) == list(other)


def _table(blob, off_ptr, n, owner=None):
    off = _arr(off_ptr, n + 1, np.int64) if n else np.zeros(1, dtype=np.int64)
    if owner is not None and off[-1]:
        raw = (C.c_char * int(off[-1])).from_address(blob)
        raw._owner = owner
        return StringTable(memoryview(raw).cast("B"), off)
    return StringTable(C.string_at(blob, int(off[-1])) if off[-1] else b"", off)


class LociCodes:
    """Per-locus codes "start:end:strand" (utils.py:312) of natively parsed loci, formatted
    only when a per-locus list is asked for (the TSV writer takes the per-contig fields
    the parser joined, HostBatch.loci_fields).  Slices stay lazy."""

    def __init__(self, start, end, strands):
        self._s, self._e, self._st = start, end, strands
        self._list = None

    def __len__(self):
        return len(self._s)

    def _all(self):
        if self._list is None:
            st = self._st
            self._list = ["{}:{}:{}".format(a, b, st[i]) for i, (a, b) in
                          enumerate(zip(self._s.tolist(), self._e.tolist()))]
        return self._list

    def __getitem__(self, i):
        if isinstance(i, slice):
            a, b, step = i.indices(len(self))
            if step == 1:
                return LociCodes(self._s[a:b], self._e[a:b], _Sliced(self._st, a, b))
            return self._all()[i]
        return self._all()[i]

    def __iter__(self):
        return iter(self._all())

    def __eq__(self, other):
        return list(self._all()) == list(other)


class _Sliced:
    def __init__(self, table, a, b):
        self._t, self._a, self._n = table, a, b - a

    def __len__(self):
        return self._n

    def __getitem__(self, i):
        return self._t[self._a + i]


def _strings(blob, off_ptr, n):
    if n == 0:
        return []
    off = _arr(off_ptr, n + 1, np.int64)
    raw = C.string_at(blob, int(off[-1])) if off[-1] else b""
    text = raw.decode("ascii")
    return [text[off[i]:off[i + 1]] for i in range(n)]


def parse(contigs_path, blastout_path, gff_path, edges, min_gene_length, threads=0, warn=None):
    """-> (HostBatch, TaxonomyTables), or raises Fallback."""
    from .inputs import HostBatch
    so = load()
    h = so.wf_ingest_new()
    if not h:
        raise MemoryError("wf_ingest_new failed")
    owner = _Owner(so, h)       # frees the parse when the last array view is gone
    try:
        rc = so.wf_ingest_parse(h, os.fsencode(contigs_path), os.fsencode(blastout_path),
                                os.fsencode(gff_path), float(min_gene_length), int(threads))
        msg = so.wf_ingest_last_error(h).decode("utf-8", "replace")
        if rc in (INGEST_FALLBACK, INGEST_E_IO):   # the Python reader reports it
            raise Fallback(msg)
        if rc != INGEST_OK:
            raise IngestError("wf_ingest_parse: {} ({})".format(rc, msg))
        v = WfIngestView()
        if so.wf_ingest_get_view(h, C.byref(v)) != INGEST_OK:
            raise IngestError("wf_ingest_get_view failed")
        N, H, L = v.n_contigs, v.n_hits, v.n_loci
        if warn:   # same order as the Python reader: GFF groups, then BLAST groups
            for name in _strings(v.warn_gff_blob, v.warn_gff_off, v.n_warn_gff):
                warn("  Unknown contig in <gff> file", name)
            for name in _strings(v.warn_blast_blob, v.warn_blast_off, v.n_warn_blast):
                warn("  Unknown contig in <blastout> file", name)
        names = _strings(v.contig_blob, v.contig_off, N)
        taxa = _strings(v.taxa_blob, v.taxa_off, v.n_taxa)
        systems = _strings(v.system_blob, v.system_off, v.n_systems)
        S = max(1, v.n_systems)
        tax = TaxonomyTables(edges, extra_names=set(taxa))
        tmap = np.array([tax.index[t] for t in taxa], dtype=np.int32)
        hit_taxon_local = _arr(v.hit_taxon, H, np.int32, owner)
        # value ids index one table shared by every system
        values = _table(v.value_blob, v.value_off, v.n_values, owner)
        value_ids = _arr(v.hit_value, H * S, np.int32, owner).reshape(H, S)
        loc_start = _arr(v.loc_start, L, np.int32, owner)
        loc_end = _arr(v.loc_end, L, np.int32, owner)
        strands = _table(v.loc_strand_blob, v.loc_strand_off, L, owner)
        batch = HostBatch(
            contig_names=names, contig_lengths=_arr(v.contig_length, N, np.int64, owner),
            hit_off=_arr(v.hit_off, N + 1, np.int64, owner),
            hit_qlo=_arr(v.hit_qlo, H, np.int32, owner), hit_qhi=_arr(v.hit_qhi, H, np.int32, owner),
            hit_taxon=tmap[hit_taxon_local] if H else np.zeros(0, dtype=np.int32),
            hit_strand=_arr(v.hit_strand, H, np.int8, owner),
            hit_score=_arr(v.hit_score, H, np.float64, owner),
            hit_scov=_arr(v.hit_scov, H, np.float64, owner),
            hit_sysmask=_arr(v.hit_sysmask, H, np.uint32, owner),
            loc_off=_arr(v.loc_off, N + 1, np.int64, owner), loc_start=loc_start, loc_end=loc_end,
            loc_strand=_arr(v.loc_strand, L, np.int8, owner),
            loc_codes=LociCodes(loc_start, loc_end, strands), systems=systems,
            annot_value_ids=value_ids, annot_values=[values] * len(systems),
            hit_row=_arr(v.hit_row, H, np.int64, owner),
            loci_fields=_table(v.loci_blob, v.loci_off, N, owner),
            hit_group=_arr(v.hit_group, H, np.int32, owner) if v.hit_group else None)
        return batch, tax
    except BaseException:
        owner.__del__()
        raise
