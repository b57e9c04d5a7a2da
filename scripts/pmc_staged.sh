# SQ / memory counters for the staged kernels on cfg2 (separate --pmc passes)
set -u
O=${1:-gpurun_out/pmc_staged}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/sq -o run --output-format csv -- python3 bench.py --cpu-sample 0 --steps 2 --warmup 1 --mode staged > $O/sq.json 2> $O/sq.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 bench.py --cpu-sample 0 --steps 2 --warmup 1 --mode staged > $O/fetch.json 2> $O/fetch.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d $O/tcc -o run --output-format csv -- python3 bench.py --cpu-sample 0 --steps 2 --warmup 1 --mode staged > $O/tcc.json 2> $O/tcc.err || echo "tcc pass failed (counter names?)"
echo done
