# The k2 leg's VALU file: SQ counters of the cfg5 6,250-contig share (one --pmc group,
# kernel trace only) -> k2_pmc.json (scripts/pmc_k2.py) -> profiles/r04/k2_pmc.json, which
# bench.py's k2 leg reads (--k2-pmc-json).  OUT names gpurun_out/<OUT>.
set -u
O=gpurun_out/${OUT:-r4k2}; mkdir -p $O
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
B5="--config cfg5 --contigs 6250 --k2-contigs 0 --cpu-sample 0 --e2e= --pcie 0 --steps 3 --warmup 1"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $SQ -d $O/sq5 -o run --output-format csv -- python3 bench.py $B5 > $O/sq5.json 2> $O/sq5.err || exit $?
python3 scripts/pmc_sq_table.py $O/sq5 > $O/sq5_table.txt 2>&1
python3 scripts/pmc_k2.py $O/sq5 4 6250 $O/k2_pmc.json > $O/k2_pmc.log 2>&1
echo k2-pmc-done
