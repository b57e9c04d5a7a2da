# Round-2 GPU session b: all -m gpu tests (incl. junctions), the host-ASan C-ABI driver,
# the cfg5 explain_two profile (kernel trace + VALU counters), cfg4 PMC traffic passes,
# then the default bench line.  OUT names gpurun_out/<OUT>.
set -u
O=gpurun_out/${OUT:-r2b}; mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --cpu-sample 0 --e2e '' --pcie 0"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 timeout -k 10 300 tests/sanitize/api_driver_asan > $O/asan.log 2>&1 || { echo "asan driver failed"; tail -30 $O/asan.log; exit 1; }
tail -2 $O/asan.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_cfg5 -o run --output-format csv -- python3 bench.py --config cfg5 --cpu-sample 0 --e2e "" --pcie 0 --steps 2 --warmup 1 > $O/bench_cfg5.json 2> $O/prof_cfg5.err || { echo "cfg5 prof failed"; tail -20 $O/prof_cfg5.err; exit 1; }
timeout -s KILL 600 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS -d $O/pmc_cfg5 -o run --output-format csv -- python3 bench.py --config cfg5 --cpu-sample 0 --e2e "" --pcie 0 --steps 1 --warmup 0 > $O/pmc_cfg5.json 2> $O/pmc_cfg5.err || { echo "cfg5 pmc failed"; tail -20 $O/pmc_cfg5.err; exit 1; }
timeout -s KILL 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --cpu-sample 0 --e2e "" --pcie 0 --steps 1 --warmup 0 > $O/pmc_fetch.json 2> $O/pmc_fetch.err || { echo "fetch pmc failed"; tail -20 $O/pmc_fetch.err; exit 1; }
timeout -s KILL 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 bench.py --cpu-sample 0 --e2e "" --pcie 0 --steps 1 --warmup 0 > $O/pmc_write.json 2> $O/pmc_write.err || { echo "write pmc failed"; tail -20 $O/pmc_write.err; exit 1; }
timeout -s KILL 600 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES -d $O/pmc_valu -o run --output-format csv -- python3 bench.py --cpu-sample 0 --e2e "" --pcie 0 --steps 1 --warmup 0 > $O/pmc_valu.json 2> $O/pmc_valu.err || { echo "valu pmc failed"; tail -20 $O/pmc_valu.err; exit 1; }
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
echo done
