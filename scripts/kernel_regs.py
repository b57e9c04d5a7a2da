"""Per-kernel register / scratch / LDS table of one source file, from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (compile only, no GPU needed).

    python scripts/kernel_regs.py waafle_amd/csrc/wf_fast.hip [-DNAME ...]
"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from waafle_amd import build  # noqa: E402


def main():
    src, defs = sys.argv[1], sys.argv[2:]
    flags = [f for f in build.FLAGS if f != "-shared"]
    cmd = [build.hipcc()] + flags + defs + ["-c", src, "-o", "/tmp/kernel_regs.o",
                                            "-Rpass-analysis=kernel-resource-usage"]
    err = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in err.splitlines():
        m = re.search(r"remark: +(.*?) \[-Rpass", line)
        if not m:
            continue
        k, _, v = m.group(1).partition(":")
        k, v = k.strip(), v.strip()
        if k == "Function Name":
            cur = {"name": subprocess.run(["c++filt", v],
                                          capture_output=True, text=True).stdout.strip()}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    for r in rows:
        name = r["name"].replace("(anonymous namespace)::", "").replace("void ", "")
        name = re.sub(r"\(.*", "", name)
        print("{:48s} vgpr {:>4s} agpr {:>3s} sgpr {:>3s} spill {:>3s} scratch {:>4s} lds {:>6s} occ {:>2s}".format(
            name[:48], r.get("VGPRs", "?"), r.get("AGPRs", "?"), r.get("SGPRs", "?"),
            r.get("VGPRs Spill", "?"), r.get("ScratchSize [bytes/lane]", "?"),
            r.get("LDS Size [bytes/block]", "?"), r.get("Occupancy [waves/SIMD]", "?")))


if __name__ == "__main__":
    main()
