# Per-phase cost of the level-0 kernel by difference: the same cfg4 sample under each
# diagnostic variant (WF_SKIP builds, waafle_amd/libwaafle_hip_<name>.so), kernel trace only.
set -u
O=gpurun_out/${OUT:-var}; mkdir -p $O
export TMPDIR=/tmp
# heartbeat: a long profiled run prints nothing until it ends
(while sleep 45; do echo "heartbeat $(date +%T)"; done) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for v in ${VARIANTS}; do
  lib=waafle_amd/libwaafle_hip.so; [ "$v" != base ] && lib=waafle_amd/libwaafle_hip_$v.so
  WAAFLE_HIP_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 bench.py --cpu-sample 0 --e2e= --pcie 0 --contigs ${NC:-200000} --steps 3 --warmup 1 > $O/$v.json 2> $O/$v.err || { echo "$v failed"; tail -5 $O/$v.err; exit 1; }
  echo "$v: $(python3 scripts/show_prof.py $O/$v/run_kernel_stats.csv | grep k_wave0)"
done
