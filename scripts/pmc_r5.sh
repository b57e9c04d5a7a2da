# Round-5 counter passes over the cfg4 bench (one --pmc group per run, kernel trace only;
# MI355X_MICROARCH.md HBM/rocprofv3 section): FETCH_SIZE and WRITE_SIZE in separate runs ->
# traffic_cfg4.json (whole pass + the dominant kernel); SQ instruction/wave counters ->
# cfg4_valu.json (pmc_main.py) + a per-kernel table; instruction-cache counters (ICACHE=1).
# OUT names gpurun_out/<OUT>.
set -u
O=gpurun_out/${OUT:-r5pmc}; mkdir -p $O
export TMPDIR=/tmp
B4="--k2-contigs 0 --cpu-sample 0 --e2e= --pcie 0 --shares= --steps 3 --warmup 1"
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
IC="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"
if [ "${TRAFFIC:-1}" = 1 ]; then
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch4 -o run --output-format csv -- python3 bench.py $B4 > $O/fetch4.json 2> $O/fetch4.err || exit $?
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/write4 -o run --output-format csv -- python3 bench.py $B4 > $O/write4.json 2> $O/write4.err || exit $?
  python3 scripts/traffic.py $O/fetch4 $O/write4 cfg4 1000000 $O/traffic_cfg4.json --pass 4 --dominant ${DOM:-k_triage} > $O/traffic.log 2>&1 || echo "traffic parse failed" >> $O/traffic.log
fi
if [ "${SQPASS:-1}" = 1 ]; then
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $SQ -d $O/sq4 -o run --output-format csv -- python3 bench.py $B4 > $O/sq4.json 2> $O/sq4.err || exit $?
  python3 scripts/pmc_sq_table.py $O/sq4 > $O/sq4_table.txt 2>&1
  python3 scripts/pmc_main.py $O/sq4 4 cfg4 1000000 $O/cfg4_valu.json ${DOM:-k_triage} > $O/valu.log 2>&1 || echo "valu parse failed" >> $O/valu.log
fi
if [ "${ICACHE:-0}" = 1 ]; then
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $IC -d $O/ic4 -o run --output-format csv -- python3 bench.py $B4 > $O/ic4.json 2> $O/ic4.err || exit $?
  python3 scripts/pmc_sq_table.py $O/ic4 > $O/ic4_table.txt 2>&1
fi
echo pmc-done
