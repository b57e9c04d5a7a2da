# Round-5 k2-leg counters (the cfg5 6,250-contig share, one --pmc group per run, kernel trace
# only; MI355X_MICROARCH.md HBM/rocprofv3 section): SQ counters -> k2_pmc.json (pmc_k2.py,
# read by bench.py's k2 leg), FETCH_SIZE and WRITE_SIZE in separate runs -> traffic_cfg5.json
# (per kernel; k_big_sparse = the explain_two kernel).  OUT names gpurun_out/<OUT>.
set -u
O=gpurun_out/${OUT:-r5k2}; mkdir -p $O
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
B5="--config cfg5 --contigs 6250 --k2-contigs 0 --cpu-sample 0 --e2e= --pcie 0 --shares= --steps 3 --warmup 1"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $SQ -d $O/sq5 -o run --output-format csv -- python3 bench.py $B5 > $O/sq5.json 2> $O/sq5.err || exit $?
python3 scripts/pmc_sq_table.py $O/sq5 > $O/sq5_table.txt 2>&1
python3 scripts/pmc_k2.py $O/sq5 4 6250 $O/k2_pmc.json > $O/k2_pmc.log 2>&1
if [ "${TRAFFIC:-1}" = 1 ]; then
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch5 -o run --output-format csv -- python3 bench.py $B5 > $O/fetch5.json 2> $O/fetch5.err || exit $?
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/write5 -o run --output-format csv -- python3 bench.py $B5 > $O/write5.json 2> $O/write5.err || exit $?
  python3 scripts/traffic.py $O/fetch5 $O/write5 cfg5 6250 $O/traffic_cfg5.json --pass 4 --dominant k_big_sparse > $O/traffic5.log 2>&1 || echo "traffic parse failed" >> $O/traffic5.log
fi
echo k2-pmc-done
