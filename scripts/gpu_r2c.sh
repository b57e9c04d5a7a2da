# Round-2 GPU session c: all -m gpu tests, the host-ASan C-ABI driver, smoke, then the
# default (cfg4) bench line.  OUT names gpurun_out/<OUT>.  Each GPU step has its own limit;
# the chain stops at the first failure.
set -u
O=gpurun_out/${OUT:-r2c}; mkdir -p $O
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
fi
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 timeout -k 10 200 tests/sanitize/api_driver_asan > $O/asan.log 2>&1 || { echo "asan driver failed"; tail -30 $O/asan.log; exit 1; }
tail -2 $O/asan.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
echo done
