# PMC passes on the level-0 kernel at a cfg4 sample (OUT names gpurun_out/<OUT>): the SQ
# issue/wait picture, then the VALU mix.  One counter group per run (rocprofv3 does not split).
set -u
O=gpurun_out/${OUT:-pmcf}; mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --cpu-sample 0 --e2e= --pcie 0 --contigs ${NC:-200000} --steps 1 --warmup 0"
timeout -s KILL 120 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -iE "SQ_INSTS_VALU|F64|SQ_ACTIVE|SQ_WAIT|SQ_BUSY|LDS_BANK|SQ_INST_CYCLES" $O/avail.txt | head -80 > $O/avail_sq.txt || true
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/sq -o run --output-format csv -- $B > $O/sq.json 2> $O/sq.err || { echo "sq pmc failed"; tail -20 $O/sq.err; exit 1; }
echo done
