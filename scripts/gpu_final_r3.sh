# Round-3 measurement session: the default bench line (CPU legs included), kernel-trace stats
# of cfg4 and of the cfg5 6,250-contig share, then the PMC passes (scripts/pmc_r3.sh).
# OUT names gpurun_out/<OUT>.
set -u
O=gpurun_out/${OUT:-r3f}; mkdir -p $O
export TMPDIR=/tmp
SKIP_TESTS=1 OUT=${OUT:-r3f} bash scripts/gpu_r3.sh || exit $?
python3 scripts/show_prof.py $O/prof4/run_kernel_stats.csv > $O/prof4.txt 2>&1
python3 scripts/show_prof.py $O/prof5/run_kernel_stats.csv > $O/prof5.txt 2>&1
OUT=${OUT:-r3f}/pmc bash scripts/pmc_r3.sh || exit $?
echo final-done
