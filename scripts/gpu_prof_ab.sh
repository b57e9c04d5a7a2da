# Parity tests, then a rocprofv3 kernel-trace summary of the cfg2 bench per variant.
# VARIANTS: ';'-separated env assignments; ROUND names gpurun_out/<ROUND>.
set -u
O=gpurun_out/${ROUND:-profab}; mkdir -p $O
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
  echo "pytest rc=$rc" >> $O/gpu_tests.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
IFS=';' read -ra VS <<< "${VARIANTS:-WF_AB=0}"
for v in "${VS[@]}"; do
  tag=$(echo $v | tr ' =' '__')
  for kv in $v; do export "$kv"; done
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_$tag -o run --output-format csv -- python3 bench.py --cpu-sample 0 --steps 10 --config ${CFG:-cfg2} > $O/bench_$tag.json 2> $O/prof_$tag.err || exit $?
  python scripts/show_prof.py $O/prof_$tag/run_kernel_stats.csv > $O/prof_$tag.txt 2>&1 || true
  for kv in $v; do unset "${kv%%=*}"; done
done
echo done
