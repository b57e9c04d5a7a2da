# Round-2 GPU session e: profiles of the default cfg4 pass (kernel trace + stats, FETCH_SIZE
# and WRITE_SIZE PMC passes, SQ counters) and of the explain_two (k2) kernels on cfg5 (NC5
# stress contigs, default 30,000: the whole 50,000 exceed one wf_score call's 32-bit
# attachment-leaf indices; GpuScorer.score splits such batches, bench.py times one call).
# OUT names gpurun_out/<OUT>.  Every GPU step has its own limit; the chain stops at the
# first failure.  Post-processing (traffic.py, k2_roofline.py) runs on the CPU afterwards.
set -u
O=gpurun_out/${OUT:-r2e}; mkdir -p $O
export TMPDIR=/tmp
(while sleep 45; do echo "heartbeat $(date +%T)" >> $O/heartbeat.txt; done) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
B="python3 bench.py --cpu-sample 0 --e2e= --pcie 0 --k2-json="
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cfg4 -o run --output-format csv -- $B --steps 3 --warmup 1 > $O/bench_cfg4_prof.json 2> $O/prof_cfg4.err || { echo "cfg4 prof failed"; tail -20 $O/prof_cfg4.err; exit 1; }
echo prof_cfg4 ok
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- $B --steps 1 --warmup 0 > $O/pmc_fetch.json 2> $O/pmc_fetch.err || { echo "fetch pmc failed"; tail -20 $O/pmc_fetch.err; exit 1; }
echo fetch ok
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- $B --steps 1 --warmup 0 > $O/pmc_write.json 2> $O/pmc_write.err || { echo "write pmc failed"; tail -20 $O/pmc_write.err; exit 1; }
echo write ok
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/pmc_valu -o run --output-format csv -- $B --steps 1 --warmup 0 > $O/pmc_valu.json 2> $O/pmc_valu.err || { echo "valu pmc failed"; tail -20 $O/pmc_valu.err; exit 1; }
echo valu ok
K="$B --config cfg5 --contigs ${NC5:-30000}"
timeout -k 10 400 $K --steps 3 --warmup 1 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { echo "cfg5 bench failed"; tail -20 $O/bench_cfg5.err; exit 1; }
cat $O/bench_cfg5.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_cfg5 -o run --output-format csv -- $K --steps 3 --warmup 1 > $O/bench_cfg5_prof.json 2> $O/prof_cfg5.err || { echo "cfg5 prof failed"; tail -20 $O/prof_cfg5.err; exit 1; }
echo prof_cfg5 ok
timeout -s KILL 400 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES -d $O/pmc_cfg5 -o run --output-format csv -- $K --steps 3 --warmup 1 > $O/pmc_cfg5.json 2> $O/pmc_cfg5.err || { echo "cfg5 pmc failed"; tail -20 $O/pmc_cfg5.err; exit 1; }
echo done
