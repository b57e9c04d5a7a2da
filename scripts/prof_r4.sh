# Round-4 kernel-trace session: rocprofv3 --kernel-trace --stats of the cfg4 bench (and the
# cfg5 6,250-contig share with PROF5=1), per-level durations of the last pass (lvl.py), the
# first-form lap tables (stamps builds, STAMPS=1).  OUT names gpurun_out/<OUT>.
set -u
O=gpurun_out/${OUT:-r4p}; mkdir -p $O
export TMPDIR=/tmp
Q="--cpu-sample 0 --e2e= --pcie 0 --k2-contigs 0"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof4 -o run --output-format csv -- python3 bench.py $Q --steps 3 --warmup 1 ${PROF_ARGS:-} > $O/prof4.json 2> $O/prof4.err || exit $?
python3 scripts/show_prof.py $O/prof4/run_kernel_stats.csv > $O/prof4.txt 2>&1
f=$(ls $O/prof4/*kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find $O/prof4 -name "*kernel_trace.csv" | head -1)
python3 scripts/lvl.py $f > $O/prof4_levels.txt 2>&1
if [ "${PROF5:-0}" = 1 ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof5 -o run --output-format csv -- python3 bench.py --config cfg5 --contigs 6250 $Q --steps 3 --warmup 1 > $O/prof5.json 2> $O/prof5.err || exit $?
  python3 scripts/show_prof.py $O/prof5/run_kernel_stats.csv > $O/prof5.txt 2>&1
fi
if [ "${STAMPS:-0}" = 1 ]; then
  for v in stamps stampsroll; do
    WAAFLE_HIP_LIB=waafle_amd/libwaafle_hip_$v.so timeout -k 10 300 python scripts/wave_stamps.py > $O/$v.json 2> $O/$v.err || exit $?
  done
fi
echo prof-done
