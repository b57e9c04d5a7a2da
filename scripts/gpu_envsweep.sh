# rocprofv3 kernel-trace summaries of the cfg2 bench for a list of environment settings
# (measurement aids only).  VARIANTS: ';'-separated env assignments; ROUND names the dir.
set -u
O=gpurun_out/${ROUND:-envsweep}; mkdir -p $O
export TMPDIR=/tmp
IFS=';' read -ra VS <<< "${VARIANTS:-WF_X=0}"
for v in "${VS[@]}"; do
  tag=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_$tag -o run --output-format csv -- python3 bench.py --cpu-sample 0 --steps 5 --warmup 1 > $O/b_$tag.json 2> $O/b_$tag.err || exit $?
  python scripts/show_prof.py $O/p_$tag/run_kernel_stats.csv > $O/p_$tag.txt 2>&1 || true
done
echo done
