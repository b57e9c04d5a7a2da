# Round-2 GPU session: parity tests, smoke, the cfg4 bench line, and a kernel-trace profile
# of the cfg4 pass.  OUT names gpurun_out/<OUT>.  Every GPU step has its own time limit and
# the chain stops at the first failure.
set -u
O=gpurun_out/${OUT:-r2a}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --cpu-sample 0 --e2e "" --pcie 0 --steps 3 --warmup 1 > $O/bench_prof.json 2> $O/prof.err || { echo "prof failed"; tail -20 $O/prof.err; exit 1; }
echo done
