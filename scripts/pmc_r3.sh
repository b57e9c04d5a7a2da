# Round-3 counter passes (one --pmc group per run, kernel trace only; MI355X_MICROARCH.md
# HBM/rocprofv3 section): cfg4 FETCH_SIZE, cfg4 WRITE_SIZE -> per-pass traffic; cfg4 and
# cfg5 (6,250-contig share) SQ instruction/wave counters.  OUT names gpurun_out/<OUT>.
set -u
O=gpurun_out/${OUT:-r3pmc}; mkdir -p $O
export TMPDIR=/tmp
B4="--k2-contigs 0 --cpu-sample 0 --e2e= --pcie 0 --steps 3 --warmup 1"
B5="--config cfg5 --contigs 6250 --k2-contigs 0 --cpu-sample 0 --e2e= --pcie 0 --steps 3 --warmup 1"
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch4 -o run --output-format csv -- python3 bench.py $B4 > $O/fetch4.json 2> $O/fetch4.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/write4 -o run --output-format csv -- python3 bench.py $B4 > $O/write4.json 2> $O/write4.err || exit $?
python3 scripts/traffic.py $O/fetch4 $O/write4 cfg4 1000000 $O/traffic_cfg4.json --pass 4 > $O/traffic.log 2>&1 || echo "traffic parse failed" >> $O/traffic.log
timeout -k 10 300 rocprofv3 --kernel-trace --pmc $SQ -d $O/sq4 -o run --output-format csv -- python3 bench.py $B4 > $O/sq4.json 2> $O/sq4.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc $SQ -d $O/sq5 -o run --output-format csv -- python3 bench.py $B5 > $O/sq5.json 2> $O/sq5.err || exit $?
python3 scripts/pmc_sq_table.py $O/sq4 > $O/sq4_table.txt 2>&1
python3 scripts/pmc_sq_table.py $O/sq5 > $O/sq5_table.txt 2>&1
python3 scripts/pmc_k2.py $O/sq5 4 6250 $O/k2_pmc.json > $O/k2_pmc.log 2>&1
echo done
