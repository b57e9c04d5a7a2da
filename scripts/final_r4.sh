# Round-4 measurement session (one gpurun call, every step under its own time limit):
#   PMC=1   counter passes of the cfg4 bench (pmc_r4.sh: FETCH/WRITE -> traffic_cfg4.json,
#           SQ -> cfg4_valu.json) and a rocprofv3 kernel-trace summary of the same command
#   BENCH=1 the full bench line (CPU legs, k2 leg, PCIe and CLI scopes)
#   N2=1    bench.py's N > 1 branch as two gloo ranks on device 0 (a rehearsal line)
# OUT names gpurun_out/<OUT>; copy what is judged into profiles/r04/.
set -u
O=gpurun_out/${OUT:-r4final}; mkdir -p $O
export TMPDIR=/tmp
Q="--cpu-sample 0 --e2e= --pcie 0 --k2-contigs 0"
if [ "${PMC:-0}" = 1 ]; then
  OUT=$(basename $O) TRAFFIC=1 SQPASS=1 bash scripts/pmc_r4.sh || exit $?
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py $Q --steps 3 --warmup 1 > $O/kt.json 2> $O/kt.err || exit $?
  python3 scripts/show_prof.py $O/kt/run_kernel_stats.csv > $O/cfg4_kernel_stats.txt 2>&1
  f=$(find $O/kt -name "*kernel_trace.csv" | head -1)
  python3 scripts/lvl.py $f > $O/cfg4_levels.txt 2>&1
fi
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python3 scripts/show_bench.py $O/bench.json
fi
if [ "${N2:-0}" = 1 ]; then
  export HSA_ENABLE_IPC_MODE_LEGACY=0
  timeout -k 10 420 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --cpu-sample 0 --e2e= --pcie 0 --backend gloo --device-map 0,0 > $O/bench_n2.json 2> $O/bench_n2.err || { tail -20 $O/bench_n2.err; exit 1; }
  python3 scripts/show_bench.py $O/bench_n2.json
fi
echo final-done
