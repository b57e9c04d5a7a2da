# round-3 GPU session: parity tests, smoke, the default bench line (cfg4 + the cfg5 k2 leg +
# CPU legs + scopes ii/iii), kernel-trace stats of cfg4 and of the cfg5 6,250-contig share.
# OUT names gpurun_out/<OUT>; TESTS selects the pytest targets; SKIP_TESTS=1: none;
# BENCH=0 skips the default bench; PROF=0 skips the profiles.
set -u
O=gpurun_out/${OUT:-r3}; mkdir -p $O
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 1500 python -u -m pytest ${TESTS:-tests} -x -q -m gpu --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || exit $?
fi
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof5 -o run --output-format csv -- python3 bench.py --config cfg5 --contigs 6250 --k2-contigs 0 --cpu-sample 0 --e2e '' --pcie 0 --steps 4 --warmup 1 > $O/prof5.json 2> $O/prof5.err || exit $?
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof4 -o run --output-format csv -- python3 bench.py --k2-contigs 0 --cpu-sample 0 --e2e '' --pcie 0 --steps 4 --warmup 1 > $O/prof4.json 2> $O/prof4.err || exit $?
fi
echo done
