"""The wave kernels' cross-lane primitives (waafle_amd/csrc/wf_lanes.h: DPP row
permutations and the CDNA4 permlane swaps instead of ds_bpermute) against __shfl_xor and a
serial scan, on the GPU (tests/lanes/lanes_check.hip, built by waafle_amd/build.py)."""
import os
import subprocess

import pytest

from waafle_amd import build

HERE = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(HERE, "lanes", "lanes_check")


def test_lanes_check_builds():
    assert build.build_lanes_check(verbose=False) == BIN and os.path.exists(BIN)


@pytest.mark.gpu
def test_lane_primitives_match_shuffles():
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.split("\n")
    assert sum(1 for x in lines if x.endswith(" ok")) == 10, r.stdout
