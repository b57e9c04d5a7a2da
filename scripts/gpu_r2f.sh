# Round-2 GPU session f: parity tests of the product library, then an A/B of library
# variants on the full cfg4 pass (kernel trace + stats each).  VARIANTS: space-separated
# TAG[:LIB[:ENV=VAL,ENV=VAL[:BENCH_ARG,BENCH_ARG]]]; LIB "base" (or empty) = waafle_amd/libwaafle_hip.so, else
# waafle_amd/libwaafle_hip_LIB.so.  OUT names gpurun_out/<OUT>.  Every GPU step has its own
# limit; the chain stops at the first failure.
set -u
O=gpurun_out/${OUT:-r2f}; mkdir -p $O
export TMPDIR=/tmp
(while sleep 45; do echo "heartbeat $(date +%T)" >> $O/heartbeat.txt; done) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -40 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
fi
for spec in ${VARIANTS:-base}; do
  IFS=':' read -r v libn envs vargs <<< "$spec"
  lib=waafle_amd/libwaafle_hip.so; [ -n "${libn:-}" ] && [ "$libn" != base ] && lib=waafle_amd/libwaafle_hip_$libn.so
  EV=""; [ -n "${envs:-}" ] && EV=$(echo "$envs" | tr ',' ' ')
  VA=""; [ -n "${vargs:-}" ] && VA=$(echo "$vargs" | tr ',' ' ')
  ( export WAAFLE_HIP_LIB=$lib $EV; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 bench.py --cpu-sample 0 --e2e= --pcie 0 --k2-json= --steps ${STEPS:-5} --warmup 1 ${BENCH_ARGS:-} $VA > $O/$v.json 2> $O/$v.err ) || { echo "$v failed"; tail -5 $O/$v.err; exit 1; }
  echo "$v: $(python3 -c "import json,sys; d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]); print(round(d['kernel_ms']['wf_score_pass'],3), 'ms/pass')")"
  python3 scripts/show_prof.py $O/$v/run_kernel_stats.csv | head -8
done
echo done
