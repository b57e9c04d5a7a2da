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


def up_to_date():
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def build(force=False, verbose=True):
    if not force and up_to_date():
        return LIB
    cmd = [hipcc()] + FLAGS + SOURCES + ["-o", LIB + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
