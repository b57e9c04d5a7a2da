# Quick GPU iteration: parity (tests/test_gpu_parity.py unless TESTS is set), the wave-form
# stamps (diagnostic library) and a cfg4 bench without the CPU legs.  OUT names gpurun_out/<OUT>.
set -u
O=gpurun_out/${OUT:-q}; mkdir -p $O
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
fi
if [ "${STAMPS:-1}" = 1 ]; then
  WAAFLE_HIP_LIB=waafle_amd/libwaafle_hip_stamps.so timeout -k 10 300 python scripts/wave_stamps.py > $O/stamps.json 2> $O/stamps.err || exit $?
fi
timeout -k 10 300 python bench.py --cpu-sample 0 --e2e= --pcie 0 ${BENCH_ARGS:---k2-contigs 0} > $O/bench.json 2> $O/bench.err || exit $?
python scripts/show_bench.py $O/bench.json
