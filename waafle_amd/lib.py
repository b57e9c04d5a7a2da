"""ctypes binding of libwaafle_hip.so (include/waafle_hip.h).

The product path has no CPU fallback: if the in-tree library is missing or cannot be
loaded, `load()` raises.  Build it with `python -m waafle_amd.build`.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libwaafle_hip.so")

WF_OK, WF_E_BADINPUT, WF_E_HIP, WF_E_RUNAWAY, WF_E_NOMEM, WF_E_STATE, WF_E_EMPTYMASK, WF_E_TOOBIG = \
    0, -1, -2, -3, -4, -5, -6, -7
CALL_UNCLASSIFIED, CALL_NO_LGT, CALL_LGT = 0, 1, 2
MODE_STAGED = 0
MODE_LEVEL0 = 2
MODE_WAVES = 3
OPT_SPARSE_BIG, OPT_ATT_LIMIT, OPT_WAVE_TWO, OPT_DUMP_CAP, OPT_TRIAGE = 1, 2, 3, 4, 5   # wf_set_option
PHASES = ("waves", "attach", "segments", "decide", "big", "handover", "rollup", "triage")   # wf_phase 0..7
N_PHASES = 8
ABI_VERSION = 6

_P = C.c_void_p


class WfTaxonomy(C.Structure):
    _fields_ = [("n", C.c_int32), ("parent", _P), ("depth", _P), ("sib_parent", _P),
                ("leaf_count", _P), ("root", C.c_int32), ("unknown", C.c_int32)]


class WfParams(C.Structure):
    _fields_ = [("k1", C.c_double), ("k2", C.c_double), ("range", C.c_double),
                ("min_overlap", C.c_double), ("min_scov", C.c_double),
                ("ambiguous_fraction", C.c_double), ("disambiguate_one", C.c_int32),
                ("disambiguate_two", C.c_int32), ("jump_taxonomy", C.c_int32),
                ("allow_lca", C.c_int32), ("ambiguous_threshold", C.c_int32),
                ("sister_penalty", C.c_int32), ("clade_genes", C.c_int32),
                ("clade_leaves", C.c_int32), ("weak_loci", C.c_int32),
                ("annotation_threshold", C.c_int32), ("stranded", C.c_int32)]


class WfBatch(C.Structure):
    _fields_ = [("n_contigs", C.c_int32), ("n_systems", C.c_int32), ("n_hits", C.c_int64),
                ("n_loci", C.c_int64), ("max_hits", C.c_int32), ("max_loci", C.c_int32),
                ("device_resident", C.c_int32), ("_pad", C.c_int32),
                ("hit_off", _P), ("hit_qlo", _P), ("hit_qhi", _P), ("hit_taxon", _P),
                ("hit_strand", _P), ("hit_score", _P), ("hit_scov", _P), ("hit_sysmask", _P),
                ("loc_off", _P), ("loc_start", _P), ("loc_end", _P), ("loc_strand", _P),
                ("hit_key", _P)]


class WfResult(C.Structure):
    _fields_ = [("call", _P), ("crit", _P), ("rank", _P), ("clade1", _P), ("clade2", _P),
                ("direction", _P), ("iterations", _P), ("synteny", _P), ("n_meld1", _P),
                ("n_meld2", _P), ("meld", _P), ("annot_hit", _P), ("pair_evals", _P),
                ("status", _P), ("need_bytes", _P), ("ppot_sum", _P)]


class WfTiming(C.Structure):
    _fields_ = [("pass_ms", C.c_double), ("passes", C.c_int64),
                ("phase_ms", C.c_double * N_PHASES), ("phase_spans", C.c_int64 * N_PHASES)]

    def phases(self):
        """{phase name: (ms summed over the timed passes, timed spans)}"""
        return {n: (float(self.phase_ms[i]), int(self.phase_spans[i])) for i, n in enumerate(PHASES)}


class WfGcBatch(C.Structure):
    _fields_ = [("n_groups", C.c_int32), ("device_resident", C.c_int32), ("n_hits", C.c_int64),
                ("hit_off", _P), ("hit_qlo", _P), ("hit_qhi", _P), ("hit_strand", _P),
                ("hit_scov", _P)]


class WfGcParams(C.Structure):
    _fields_ = [("min_overlap", C.c_double), ("min_scov", C.c_double),
                ("min_gene_length", C.c_double), ("stranded", C.c_int32), ("_pad", C.c_int32)]


class WfGcResult(C.Structure):
    _fields_ = [("n_genes", _P), ("gene_start", _P), ("gene_stop", _P), ("gene_strand", _P)]


class WfJnBatch(C.Structure):
    _fields_ = [("n_contigs", C.c_int32), ("device_resident", C.c_int32), ("n_pairs", C.c_int64),
                ("n_loci", C.c_int64), ("contig_length", _P), ("loc_off", _P), ("loc_start", _P),
                ("loc_end", _P), ("pair_contig", _P), ("m1_start", _P), ("m1_end", _P),
                ("m2_start", _P), ("m2_end", _P)]


class WfJnParams(C.Structure):
    _fields_ = [("min_overlap_sites", C.c_int64)]


class WfJnResult(C.Structure):
    _fields_ = [("junction_hits", _P), ("coverage_gene1", _P), ("coverage_gene2", _P),
                ("coverage_junction", _P), ("ratio", _P), ("locus_hits", _P), ("coverage", _P),
                ("pair_first", _P), ("pair_mask", _P)]


class WfDetails(C.Structure):
    _fields_ = [("n_evals", C.c_int64), ("eval_contig", _P), ("eval_level", _P),
                ("n_segs", C.c_int64), ("seg_level", _P), ("seg_contig", _P), ("seg_clade", _P),
                ("seg_locus", _P), ("seg_mean", _P), ("seg_nspan", _P), ("span_off", _P),
                ("spans", _P)]


# every symbol the header declares, with its ctypes signature
SIGNATURES = {
    "wf_abi_version": (C.c_int, []),
    "wf_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "wf_init": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "wf_free": (None, [C.c_void_p]),
    "wf_last_error": (C.c_char_p, [C.c_void_p]),
    "wf_set_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "wf_set_lds_bytes": (C.c_int, [C.c_void_p, C.c_int64]),
    "wf_set_mode": (C.c_int, [C.c_void_p, C.c_int]),
    "wf_set_option": (C.c_int, [C.c_void_p, C.c_int, C.c_int64]),
    "wf_set_taxonomy": (C.c_int, [C.c_void_p, C.POINTER(WfTaxonomy)]),
    "wf_score": (C.c_int, [C.c_void_p, C.POINTER(WfBatch), C.POINTER(WfParams),
                           C.POINTER(WfResult)]),
    "wf_pack_hit_keys": (C.c_int, [C.c_int64, _P, _P, _P, _P, C.c_double, _P]),
    "wf_synchronize": (C.c_int, [C.c_void_p]),
    "wf_timing_enable": (C.c_int, [C.c_void_p, C.c_int]),
    "wf_timing_read": (C.c_int, [C.c_void_p, C.POINTER(WfTiming)]),
    "wf_genecall": (C.c_int, [C.c_void_p, C.POINTER(WfGcBatch), C.POINTER(WfGcParams),
                              C.POINTER(WfGcResult)]),
    "wf_junctions": (C.c_int, [C.c_void_p, C.POINTER(WfJnBatch), C.POINTER(WfJnParams),
                               C.POINTER(WfJnResult)]),
    "wf_details_enable": (C.c_int, [C.c_void_p, C.c_int]),
    "wf_details_read": (C.c_int, [C.c_void_p, C.POINTER(WfDetails)]),
}

_lib = None


class WaafleHipError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("libwaafle_hip error {}: {}".format(code, msg))
        self.code = code
        self.msg = msg

    def __reduce__(self):   # picklable across ranks (keeps the failing contig indices)
        return (type(self), (self.code, self.msg), {"contigs": getattr(self, "contigs", ())})


def load(path=None):
    """Load the in-tree HIP library (raises if it is absent -- no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    # WAAFLE_HIP_LIB: a diagnostic build variant (python -m waafle_amd.build --variant=...)
    path = path or os.environ.get("WAAFLE_HIP_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise ImportError("{} not built: run `python -m waafle_amd.build` "
                          "(the MI355X path has no CPU fallback)".format(path))
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.wf_abi_version() != ABI_VERSION:
        raise ImportError("libwaafle_hip ABI mismatch")
    _lib = lib
    return lib


def device_count():
    lib = load()
    n = C.c_int(0)
    lib.wf_device_count(C.byref(n))
    return n.value


def pack_hit_keys(taxon, strand, scov, sysmask, min_scov):
    """wf_batch.hit_key (include/waafle_hip.h, wf_pack_hit_keys' layout) in numpy: taxon |
    (scov >= min_scov) << 24 | (strand == 1) << 25 | (sysmask & 63) << 26."""
    key = np.asarray(taxon).astype(np.uint32)
    key |= (np.asarray(scov) >= min_scov).astype(np.uint32) << np.uint32(24)
    key |= (np.asarray(strand) == 1).astype(np.uint32) << np.uint32(25)
    key |= (np.asarray(sysmask).astype(np.uint32) & np.uint32(63)) << np.uint32(26)
    return key


def ptr(a):
    """Host numpy array -> void* (array must stay alive for the call)."""
    return a.ctypes.data_as(C.c_void_p) if a is not None else None
