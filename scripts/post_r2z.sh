# Copy the closing session's results (gpurun_out/$1, default r2z) into profiles/ (v5).
set -eu
I=gpurun_out/${1:-r2z}
P=profiles
tail -1 $I/bench.json > $P/r02_bench_cfg4_v6.json
python3 scripts/traffic.py $I/pmc_fetch $I/pmc_write cfg4 1000000 $P/r02_traffic_cfg4.json --pass 1 > /dev/null
cp $I/prof_cfg4/run_kernel_stats.csv $P/r02_cfg4_kernel_stats_v6.csv
python3 scripts/show_prof.py $P/r02_cfg4_kernel_stats_v6.csv > $P/r02_cfg4_kernel_stats_v6_summary.txt || true
tail -1 $I/bench_cfg4_prof.json > $P/r02_bench_cfg4_prof_v6.json
cp $I/prof_cfg5/run_kernel_stats.csv $P/r02_cfg5_kernel_stats_v6.csv
python3 scripts/show_prof.py $P/r02_cfg5_kernel_stats_v6.csv > $P/r02_cfg5_kernel_stats_v6_summary.txt || true
tail -1 $I/bench_cfg5.json > $P/r02_bench_cfg5_30k_v6.json
python3 scripts/k2_roofline.py $I/bench_cfg5_prof.json $I/prof_cfg5/run_kernel_stats.csv 4 $P/r02_k2_cfg5.json --pmc $I/pmc_cfg5 4 > /dev/null
python3 scripts/pmc_sq_table.py $I/pmc_valu > $P/r02_cfg4_pmc_sq_v6.txt
{ tail -1 $I/gpu_tests.log; tail -1 $I/asan.log; cat $I/smoke.log | grep -v amdgpu.ids; } > $P/r02_gpu_session_v6.txt
echo post done
