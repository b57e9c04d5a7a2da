"""Build libwaafle_hip.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

    python -m waafle_amd.build            # or __graft_entry__.build()
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libwaafle_hip.so")
SOURCES = [os.path.join(CSRC, "wf_kernels.hip"), os.path.join(CSRC, "wf_api.cpp")]
DEPS = SOURCES + [os.path.join(CSRC, "wf_internal.h"), os.path.join(REPO, "include", "waafle_hip.h")]

# -ffp-contract=off: no a*b+c fusion anywhere, so float64 results match numpy bit-for-bit.
FLAGS = ["--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17", "-fPIC", "-shared",
         "-Wall", "-Wno-unused-function", "-I" + os.path.join(REPO, "include"), "-I" + CSRC]


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


def build(force=False, verbose=True, stamps=False):
    """Build the product library (or, with stamps=True, the per-phase timing variant)."""
    lib = STAMPS_LIB if stamps else LIB
    if not force and up_to_date(lib):
        return lib
    extra = ["-DWF_STAMPS"] if stamps else []
    cmd = [hipcc()] + FLAGS + extra + SOURCES + ["-o", lib + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(lib + ".tmp", lib)
    return lib


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    if "--stamps" in sys.argv:
        build(force="--force" in sys.argv, stamps=True)
