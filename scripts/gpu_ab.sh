# A/B of staged variants (env toggles) on cfg2 and cfg3, after the parity tests
set -u
O=gpurun_out/${ROUND:-ab}; mkdir -p $O
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > $O/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in "WF_FLAT_ONE=1" "WF_FLAT_ONE=0" "WF_FLAT_ONE=0 WF_DEC_LDS=40960"; do
  tag=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 600 python bench.py --cpu-sample 0 > $O/cfg2_$tag.json 2> $O/cfg2_$tag.err || exit $?
  env $v timeout -k 10 600 python bench.py --config cfg3 --steps 5 --warmup 2 --cpu-sample 0 > $O/cfg3_$tag.json 2> $O/cfg3_$tag.err || exit $?
done
echo done
