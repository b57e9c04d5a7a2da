# parity tests + bench lines for cfg2 / cfg3 / cfg5 (reduced contigs for cfg5), staged and
# fused forms, plus a kernel-trace profile of the staged cfg2 run.  ROUND names the dir.
set -u
O=gpurun_out/${ROUND:-cfgs}; mkdir -p $O
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > $O/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for m in staged fused; do
  timeout -k 10 600 python bench.py --cpu-sample 0 --mode $m > $O/cfg2_$m.json 2> $O/cfg2_$m.err || exit $?
  timeout -k 10 600 python bench.py --config cfg3 --steps 5 --warmup 2 --cpu-sample 0 --mode $m > $O/cfg3_$m.json 2> $O/cfg3_$m.err || exit $?
done
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof2 -o run --output-format csv -- python3 bench.py --cpu-sample 0 --steps 5 --mode staged > $O/cfg2_prof.json 2> $O/cfg2_prof.err || exit $?
timeout -k 10 600 python bench.py --config cfg5 --contigs ${CFG5_N:-2000} --steps 3 --warmup 1 --cpu-sample 0 --mode staged > $O/cfg5_staged.json 2> $O/cfg5_staged.err || exit $?
echo done
