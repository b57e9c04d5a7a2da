# Round-6 measurement session (one gpurun call, every step under its own time limit):
#   TESTS=1 the whole GPU suite and smoke()
#   PMC=1   counter passes of the cfg4 bench (pmc_r5.sh: FETCH/WRITE -> traffic_cfg4.json,
#           SQ -> cfg4_valu.json, dominant kernel k_triage), of the cfg5 k2 leg (pmc_k2_r5.sh:
#           SQ -> k2_pmc.json, FETCH/WRITE -> traffic_cfg5.json) and rocprofv3 kernel-trace
#           summaries of the cfg4 and cfg5 commands
#   BENCH=1 the full bench line (CPU legs, k2 leg, PCIe and CLI scopes); with PMC=1 in the same
#           call it reads the counters just taken (copied into this tree's profiles/r06)
#   N2=1    bench.py's N > 1 branch as two gloo ranks on device 0 (a rehearsal line)
# OUT names gpurun_out/<OUT>; copy what is judged into profiles/r06/.
set -u
O=gpurun_out/${OUT:-r6final}; mkdir -p $O
export TMPDIR=/tmp
Q="--cpu-sample 0 --e2e= --pcie 0 --k2-contigs 0 --shares="
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if [ "${PMC:-0}" = 1 ]; then
  OUT=$(basename $O) TRAFFIC=1 SQPASS=1 bash scripts/pmc_r5.sh || exit $?
  OUT=$(basename $O) bash scripts/pmc_k2_r5.sh || exit $?
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py $Q --steps 3 --warmup 1 > $O/kt.json 2> $O/kt.err || exit $?
  python3 scripts/show_prof.py $O/kt/run_kernel_stats.csv > $O/cfg4_kernel_stats.txt 2>&1
  f=$(find $O/kt -name "*kernel_trace.csv" | head -1)
  python3 scripts/lvl.py $f > $O/cfg4_levels.txt 2>&1
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt5 -o run --output-format csv -- python3 bench.py --config cfg5 --contigs 6250 $Q --steps 3 --warmup 1 > $O/kt5.json 2> $O/kt5.err || exit $?
  python3 scripts/show_prof.py $O/kt5/run_kernel_stats.csv > $O/cfg5_6250_kernel_stats.txt 2>&1
  # (this copy of the tree: the bench step below reads this build's counters from profiles/r06)
  cp $O/traffic_cfg4.json $O/cfg4_valu.json $O/k2_pmc.json $O/traffic_cfg5.json profiles/r06/
fi
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python3 scripts/show_bench.py $O/bench.json
fi
if [ "${N2:-0}" = 1 ]; then
  export HSA_ENABLE_IPC_MODE_LEGACY=0
  timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --cpu-sample 0 --e2e= --pcie 0 --backend gloo --device-map 0,0 > $O/bench_n2.json 2> $O/bench_n2.err || { tail -20 $O/bench_n2.err; exit 1; }
  python3 scripts/show_bench.py $O/bench_n2.json
fi
echo final-done
