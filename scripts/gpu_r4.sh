# Round-4 GPU iteration: pytest -m gpu on TESTS (with -k KEXPR when set), then a cfg4 bench
# without the CPU legs (BENCH=0 skips it), both under their own time limits.
# Usage (everything on the command line, the box sees no local env):
#   gpurun -- 'OUT=r4a TESTS=tests/test_gpu_parity.py KEXPR="level0" bash scripts/gpu_r4.sh'
set -u
O=gpurun_out/${OUT:-r4}; mkdir -p $O
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  if [ -n "${KEXPR:-}" ]; then
    timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest $TESTS -x -q -m gpu -k "$KEXPR" --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  else
    timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest $TESTS -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  fi
  rc=$?
  tail -25 $O/gpu_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 300 python bench.py --cpu-sample 0 --e2e= --pcie 0 ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python scripts/show_bench.py $O/bench.json
fi
