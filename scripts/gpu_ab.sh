# A/B of staged variants (env toggles) on cfg2, cfg3 and cfg5, after the parity tests.
# VARIANTS: ';'-separated env assignments ("" = defaults); ROUND names gpurun_out/<ROUND>.
set -u
O=gpurun_out/${ROUND:-ab}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
IFS=';' read -ra VS <<< "${VARIANTS:-WF_AB=0}"
for v in "${VS[@]}"; do
  tag=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 600 python bench.py --cpu-sample 0 > $O/cfg2_$tag.json 2> $O/cfg2_$tag.err || exit $?
  env $v timeout -k 10 600 python bench.py --config cfg3 --steps 5 --warmup 2 --cpu-sample 0 > $O/cfg3_$tag.json 2> $O/cfg3_$tag.err || exit $?
  env $v timeout -k 10 600 python bench.py --config cfg5 --contigs 2000 --steps 3 --warmup 1 --cpu-sample 0 > $O/cfg5_$tag.json 2> $O/cfg5_$tag.err || exit $?
done
echo done
