# Round-2 closing GPU session: every -m gpu test, the host-ASan C-ABI driver, smoke and the
# default cfg4 bench line (gpu_r2c.sh), then the cfg4 profiles and the cfg5 k2 profile
# (gpu_r2e.sh), then cfg4 A/B variants (gpu_r2f.sh, VARIANTS).  All under gpurun_out/<OUT>.
set -u
export OUT=${OUT:-r2z}
bash scripts/gpu_r2c.sh || exit 1
bash scripts/gpu_r2e.sh || exit 1
[ -n "${VARIANTS:-}" ] && { TESTS=0 OUT=${OUT}ab bash scripts/gpu_r2f.sh || exit 1; }
echo final done
