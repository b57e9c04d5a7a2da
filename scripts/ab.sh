# Same-box A/B of library variants on the cfg4 bench (no CPU legs): VARIANTS="prod t8"
# alternates waafle_amd/libwaafle_hip.so ("prod") and libwaafle_hip_<v>.so, REPS times each.
# OUT names gpurun_out/<OUT>; each line goes to <OUT>/<v>_<rep>.json.
set -u
O=gpurun_out/${OUT:-ab}; mkdir -p $O
export TMPDIR=/tmp
Q="--cpu-sample 0 --e2e= --pcie 0 --k2-contigs ${K2:-0} --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS:-}"
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-prod}; do
    if [ "$v" = prod ]; then lib=waafle_amd/libwaafle_hip.so; else lib=waafle_amd/libwaafle_hip_$v.so; fi
    WAAFLE_HIP_LIB=$lib timeout -k 10 300 python3 bench.py $Q > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { tail -5 $O/${v}_$rep.err; exit 1; }
    echo "$v rep $rep: $(python3 scripts/show_bench.py $O/${v}_$rep.json | head -2 | tr '\n' ' ')"
  done
done
