# Iteration loop on the GPU box: GPU parity tests, then a cfg4 bench line (no CPU legs)
# and the same under a kernel trace.  OUT names gpurun_out/<OUT>; TESTS selects the pytest
# target (empty: skip the tests).
set -u
O=gpurun_out/${OUT:-iter}; mkdir -p $O
export TMPDIR=/tmp
# heartbeat: a long profiled run prints nothing until it ends
(while sleep 45; do echo "heartbeat $(date +%T)"; done) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ -n "${TESTS-tests}" ]; then
  echo "tests start $(date +%T)"
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -40 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
fi
echo "bench start $(date +%T)"
timeout -k 10 300 python3 bench.py --cpu-sample 0 --e2e= --pcie 0 ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
# ENVS: space-separated VAR=value settings, one extra bench line each (measurement aids)
for e in ${ENVS:-}; do
  env $e timeout -k 10 300 python3 bench.py --cpu-sample 0 --e2e= --pcie 0 ${BENCH_ARGS:-} > $O/bench_$e.json 2> $O/bench_$e.err || { echo "bench $e failed"; tail -20 $O/bench_$e.err; exit 1; }
  echo "$e: $(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['ms_per_step'])" $O/bench_$e.json) ms"
done
echo "prof start $(date +%T)"
timeout -k 10 170 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --cpu-sample 0 --e2e= --pcie 0 --steps 3 --warmup 1 ${BENCH_ARGS:-} > $O/bench_prof.json 2> $O/prof.err || { echo "prof failed"; tail -20 $O/prof.err; exit 1; }
echo "done $(date +%T)"
