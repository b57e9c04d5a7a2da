# PMC passes on the wave kernels at a cfg4 sample (OUT names gpurun_out/<OUT>): the SQ
# issue/wait picture, then LDS/VALU detail.  One counter group per run (rocprofv3 does not
# split groups); each pass prints a line so a long pass is not taken for a hang.
set -u
O=gpurun_out/${OUT:-pmcf}; mkdir -p $O
export TMPDIR=/tmp
# heartbeat: a long profiled run prints nothing until it ends
(while sleep 45; do echo "heartbeat $(date +%T)"; done) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
B="python3 bench.py --cpu-sample 0 --e2e= --pcie 0 --contigs ${NC:-200000} --steps 1 --warmup 0"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_INT32"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp -d $O/p$i -o run --output-format csv -- $B > $O/p$i.json 2> $O/p$i.err || { echo "pmc pass $i failed"; tail -20 $O/p$i.err; exit 1; }
  echo "pass $i done"
done
echo done
