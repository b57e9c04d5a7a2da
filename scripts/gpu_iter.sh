# One iteration on the GPU box: parity tests, cfg2/cfg3/cfg5 bench lines, and a rocprofv3
# kernel-trace summary of cfg2.  ROUND names gpurun_out/<ROUND>; SKIP_TESTS=1 skips pytest.
set -u
O=gpurun_out/${ROUND:-iter}; mkdir -p $O
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
  echo "pytest rc=$rc" >> $O/gpu_tests.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
timeout -k 10 600 python bench.py --cpu-sample 0 > $O/cfg2.json 2> $O/cfg2.err || exit $?
timeout -k 10 600 python bench.py --config cfg3 --steps 5 --warmup 2 --cpu-sample 0 > $O/cfg3.json 2> $O/cfg3.err || exit $?
timeout -k 10 600 python bench.py --config cfg5 --contigs 2000 --steps 3 --warmup 1 --cpu-sample 0 > $O/cfg5.json 2> $O/cfg5.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --cpu-sample 0 --steps 10 > $O/bench_prof.json 2> $O/prof.err || exit $?
python scripts/show_prof.py $O/prof/run_kernel_stats.csv > $O/prof.txt 2>&1 || true
python scripts/lvl.py $O/prof/run_kernel_trace.csv > $O/levels.txt 2>&1 || true
echo done
