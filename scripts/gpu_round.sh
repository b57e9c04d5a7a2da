# round-end style GPU run: parity tests, smoke, PMC traffic (two passes), bench with the
# CPU baseline, rocprofv3 kernel-trace stats.  ROUND names gpurun_out/<ROUND>.
set -u
O=gpurun_out/${ROUND:-r1}; mkdir -p $O
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu > $O/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/gpu_tests.log
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
export TMPDIR=/tmp
# traffic: 1 warmup + 3 timed passes -> 4 passes per profiled run
timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --cpu-sample 0 --steps 3 --warmup 1 > $O/pmc_fetch.json 2> $O/pmc_fetch.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 bench.py --cpu-sample 0 --steps 3 --warmup 1 > $O/pmc_write.json 2> $O/pmc_write.err || exit $?
python scripts/traffic.py $O/pmc_fetch $O/pmc_write cfg2 10000 $O/traffic_cfg2.json --pass 4 > $O/traffic.log 2>&1 || echo "traffic parse failed" >> $O/traffic.log
timeout -k 10 600 python bench.py --traffic-json $O/traffic_cfg2.json > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --cpu-sample 0 --steps 10 --traffic-json $O/traffic_cfg2.json > $O/bench_prof.json 2> $O/prof.err || exit $?
echo done
