set -u
O=gpurun_out/${OUT:-front2}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt5 -o run --output-format csv -- python3 bench.py --config cfg5 --contigs 6250 --cpu-sample 0 --e2e= --pcie 0 --shares= --k2-contigs 0 --steps 3 --warmup 1 > $O/kt5.json 2> $O/kt5.err || { tail -20 $O/kt5.err; exit 1; }
python3 scripts/show_prof.py $O/kt5/run_kernel_stats.csv > $O/cfg5_kernel_stats.txt 2>&1
f=$(find $O/kt5 -name "*kernel_trace.csv" | head -1)
python3 scripts/lvl.py $f > $O/cfg5_levels.txt 2>&1
head -12 $O/cfg5_kernel_stats.txt
head -c 3000 $O/cfg5_levels.txt
