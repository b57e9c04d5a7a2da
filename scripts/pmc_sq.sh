# SQ counters for the contig kernels on cfg2 (one --pmc pass per invocation; no tracing
# domains besides kernel dispatch).  Usage: bash scripts/pmc_sq.sh <outdir> [bench args]
set -u
O=$1; shift
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/sq -o run --output-format csv -- python bench.py --cpu-sample 0 --steps 3 --warmup 1 "$@" > $O/sq_bench.json 2> $O/sq.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU -d $O/sq2 -o run --output-format csv -- python bench.py --cpu-sample 0 --steps 3 --warmup 1 "$@" > $O/sq2_bench.json 2> $O/sq2.err || exit $?
echo done
