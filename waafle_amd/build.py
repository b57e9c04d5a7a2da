"""Build libwaafle_hip.so in-tree for gfx950 (hipcc cross-compiles without a GPU), and the
host-only native ingest library libwaafle_ingest.so (g++).

    python -m waafle_amd.build            # or __graft_entry__.build()
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libwaafle_hip.so")
SOURCES = [os.path.join(CSRC, "wf_staged.hip"), os.path.join(CSRC, "wf_fast.hip"),
           os.path.join(CSRC, "wf_triage.hip"), os.path.join(CSRC, "wf_genecall.hip"),
           os.path.join(CSRC, "wf_junctions.hip"),
           os.path.join(CSRC, "wf_api.cpp")]
DEPS = SOURCES + [os.path.join(CSRC, "wf_internal.h"), os.path.join(CSRC, "wf_device.h"),
                  os.path.join(CSRC, "wf_sparse.h"), os.path.join(CSRC, "wf_lanes.h"),
                  os.path.join(CSRC, "wf_stamps.h"),
                  os.path.join(REPO, "include", "waafle_hip.h")]

# -ffp-contract=off: no a*b+c fusion anywhere, so float64 results match numpy bit-for-bit.
FLAGS = ["--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17", "-fPIC", "-shared",
         "-Wall", "-Wno-unused-function", "-Wno-pass-failed", "-I" + os.path.join(REPO, "include"), "-I" + CSRC]


def hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.sep not in cand or os.path.exists(cand)):
            return cand
    raise RuntimeError("hipcc not found")


STAMPS_LIB = os.path.join(HERE, "libwaafle_hip_stamps.so")   # diagnostic build only


def up_to_date(lib=LIB):
    if not os.path.exists(lib):
        return False
    t = os.path.getmtime(lib)
    return all(os.path.getmtime(d) <= t for d in DEPS)


INGEST_LIB = os.path.join(HERE, "libwaafle_ingest.so")
INGEST_SOURCES = [os.path.join(CSRC, "wf_ingest.cpp")]
INGEST_DEPS = INGEST_SOURCES + [os.path.join(REPO, "include", "waafle_ingest.h")]


def build_ingest(force=False, verbose=True):
    """Host-only C++ (no HIP): the multi-threaded FASTA/BLAST/GFF parser."""
    lib = INGEST_LIB
    if not force and os.path.exists(lib) and all(
            os.path.getmtime(d) <= os.path.getmtime(lib) for d in INGEST_DEPS):
        return lib
    cxx = os.environ.get("CXX", "g++")
    cmd = [cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-Wall", "-Wextra",
           "-I" + os.path.join(REPO, "include")] + INGEST_SOURCES + ["-o", lib + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(lib + ".tmp", lib)
    return lib


def build(force=False, verbose=True, stamps=False, defines=(), out=None):
    """Build the product library (or, with stamps=True, the per-phase timing variant;
    `defines` + `out` build an experimental variant for sweeps)."""
    lib = out or (STAMPS_LIB if stamps else LIB)
    if not force and up_to_date(lib):
        return lib
    extra = (["-DWF_STAMPS"] if stamps else []) + ["-D" + d for d in defines]
    # one compile per source, in parallel, then a link step.  Objects are kept per library
    # (waafle_amd/.objs/<lib>/, git- and gpurun-ignored) and recompiled only when their
    # source or a header is newer, so an edit to one kernel file rebuilds that file alone;
    # force=True recompiles every object (e.g. after a toolchain change).
    cflags = [f for f in FLAGS if f != "-shared"]
    odir = os.path.join(HERE, ".objs", os.path.basename(lib))
    os.makedirs(odir, exist_ok=True)
    stamp = os.path.join(odir, "flags")
    flags_txt = " ".join(cflags + extra)
    same_flags = os.path.exists(stamp) and open(stamp).read() == flags_txt
    headers = [d for d in DEPS if d not in SOURCES]
    objs, procs = [], []
    for src in SOURCES:
        obj = os.path.join(odir, os.path.splitext(os.path.basename(src))[0] + ".o")
        objs.append(obj)
        if (not force and same_flags and os.path.exists(obj) and
                all(os.path.getmtime(d) <= os.path.getmtime(obj) for d in [src] + headers)):
            continue
        cmd = [hipcc()] + cflags + extra + ["-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append(subprocess.Popen(cmd))
    rcs = [p.wait() for p in procs]
    if any(rcs):
        for o in objs:                       # a failed compile leaves no stale object
            if os.path.exists(o) and not same_flags:
                os.remove(o)
        raise subprocess.CalledProcessError(max(rcs), "hipcc -c")
    with open(stamp, "w") as fh:
        fh.write(flags_txt)
    cmd = [hipcc()] + FLAGS + objs + ["-o", lib + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(lib + ".tmp", lib)
    return lib


LANES_SRC = os.path.join(REPO, "tests", "lanes", "lanes_check.hip")
LANES_BIN = os.path.join(REPO, "tests", "lanes", "lanes_check")


def build_lanes_check(force=False, verbose=True):
    """The GPU check program of the cross-lane primitives (csrc/wf_lanes.h), run by
    tests/test_gpu_lanes.py."""
    deps = [LANES_SRC, os.path.join(CSRC, "wf_lanes.h")]
    if not force and os.path.exists(LANES_BIN) and all(
            os.path.getmtime(d) <= os.path.getmtime(LANES_BIN) for d in deps):
        return LANES_BIN
    cmd = [hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-Wno-unused-result",
           "-I" + CSRC, LANES_SRC, "-o", LANES_BIN + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(LANES_BIN + ".tmp", LANES_BIN)
    return LANES_BIN


if __name__ == "__main__":
    for arg in sys.argv[1:]:
        if arg.startswith("--variant="):      # --variant=NAME:DEF1,DEF2 -> libwaafle_hip_NAME.so
            name, defs = arg.split("=", 1)[1].split(":", 1)
            build(force=True, defines=defs.split(","),
                  out=os.path.join(HERE, "libwaafle_hip_{}.so".format(name)))
            sys.exit(0)
    build(force="--force" in sys.argv)
    build_ingest(force="--force" in sys.argv)
    build_lanes_check(force="--force" in sys.argv)
    if "--stamps" in sys.argv:
        build(force="--force" in sys.argv, stamps=True)
