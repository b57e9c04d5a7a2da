# parity tests + bench + geometry sweep over the product library and a variant
set -u
O=gpurun_out/${ROUND:-sweep}; mkdir -p $O
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > $O/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/gpu_tests.log
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --cpu-sample 0 > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 600 python scripts/sweep.py ${GEOMS:+--geoms $GEOMS} > $O/sweep_product.txt 2>&1 || exit $?
if [ -n "${VARIANT:-}" ]; then
  timeout -k 10 600 python scripts/sweep.py --lib waafle_amd/libwaafle_hip_${VARIANT}.so ${GEOMS:+--geoms $GEOMS} > $O/sweep_${VARIANT}.txt 2>&1 || exit $?
fi
if [ "${STAMPS:-0}" = "1" ]; then timeout -k 10 300 python scripts/phase_stamps.py > $O/stamps.txt 2>&1 || exit $?; fi
echo done
