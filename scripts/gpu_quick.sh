# quick GPU check: parity tests + bench (no rocprof); ROUND names the output dir
set -u
O=gpurun_out/${ROUND:-quick}; mkdir -p $O
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > $O/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/gpu_tests.log
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --cpu-sample ${CPU_SAMPLE:-0} > $O/bench.json 2> $O/bench.err || exit $?
echo done
if [ "${STAMPS:-0}" = "1" ]; then timeout -k 10 300 python scripts/phase_stamps.py > $O/stamps.txt 2>&1 || exit $?; fi
