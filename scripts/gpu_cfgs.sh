# parity tests + bench lines for cfg2 / cfg3 / cfg5 (reduced contigs for cfg5)
set -u
O=gpurun_out/${ROUND:-cfgs}; mkdir -p $O
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > $O/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --cpu-sample 0 > $O/cfg2.json 2> $O/cfg2.err || exit $?
timeout -k 10 600 python bench.py --cpu-sample 0 --mode fused > $O/cfg2_fused.json 2> $O/cfg2_fused.err || exit $?
timeout -k 10 600 python bench.py --config cfg3 --steps 5 --warmup 2 --cpu-sample 0 > $O/cfg3.json 2> $O/cfg3.err || exit $?
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof2 -o run --output-format csv -- python3 bench.py --cpu-sample 0 --steps 5 > $O/cfg2_prof.json 2> $O/cfg2_prof.err || exit $?
timeout -k 10 600 python bench.py --config cfg5 --contigs ${CFG5_N:-2000} --steps 3 --warmup 1 --cpu-sample 0 > $O/cfg5.json 2> $O/cfg5.err || exit $?
echo done
