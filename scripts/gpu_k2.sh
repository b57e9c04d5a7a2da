# The isolated explain_two (k2) kernel at cfg5 (a contig sample, NC): a bench line, the same
# run under a kernel trace, a --pmc SQ_INSTS_VALU SQ_WAVES pass, then scripts/k2_roofline.py
# -> $O/k2.json.  OUT names gpurun_out/<OUT>.  Each GPU step has its own limit.
set -u
O=gpurun_out/${OUT:-k2}; mkdir -p $O
export TMPDIR=/tmp
(while sleep 45; do echo "heartbeat $(date +%T)"; done) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
ARGS="--config cfg5 --contigs ${NC:-10000} --cpu-sample 0 --cpu-shard 0 --e2e= --pcie 0 --k2-json="
echo "bench start $(date +%T)"
timeout -k 10 400 python3 bench.py $ARGS --steps 3 --warmup 1 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
echo "trace start $(date +%T)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py $ARGS --steps 3 --warmup 1 > $O/bench_prof.json 2> $O/prof.err || { echo "trace failed"; tail -20 $O/prof.err; exit 1; }
echo "pmc start $(date +%T)"
timeout -s KILL 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d $O/pmc -o run --output-format csv -- python3 bench.py $ARGS --steps 3 --warmup 1 > $O/bench_pmc.json 2> $O/pmc.err || { echo "pmc failed"; tail -20 $O/pmc.err; exit 1; }
python3 scripts/k2_roofline.py $O/bench_prof.json $O/prof/run_kernel_stats.csv 4 $O/k2.json --pmc $O/pmc 4
python3 scripts/show_prof.py $O/prof/run_kernel_stats.csv | head -20
echo "done $(date +%T)"
