# instruction-cache and wave-state counters for the contig kernel (separate --pmc passes)
set -u
O=${1:-gpurun_out/icache}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH -d $O/ic -o run --output-format csv -- python3 bench.py --cpu-sample 0 --steps 3 --warmup 1 > $O/ic.json 2> $O/ic.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/sq -o run --output-format csv -- python3 bench.py --cpu-sample 0 --steps 3 --warmup 1 > $O/sq.json 2> $O/sq.err || exit $?
echo done
