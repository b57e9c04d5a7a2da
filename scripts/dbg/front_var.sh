# kernel traces of the cfg5 bench under library variants (VARS="name ..." -> waafle_amd/libwaafle_hip_<name>.so)
set -u
O=gpurun_out/${OUT:-fvar}; mkdir -p $O
export TMPDIR=/tmp
for v in $VARS; do
  L=waafle_amd/libwaafle_hip_$v.so; [ "$v" = main ] && L=waafle_amd/libwaafle_hip.so
  WAAFLE_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 bench.py --config cfg5 --contigs 6250 --cpu-sample 0 --e2e= --pcie 0 --shares= --k2-contigs 0 --steps 3 --warmup 1 > $O/$v.json 2> $O/$v.err || { tail -20 $O/$v.err; exit 1; }
  f=$(find $O/$v -name "*kernel_trace.csv" | head -1)
  echo "== $v $(python3 scripts/show_bench.py $O/$v.json | head -1 | cut -c1-80)"
  python3 scripts/lvl.py $f | tr '|' '\n' | grep -E "k_front|k_sort|k_seg_build|k_seg_rec|k_big" | tr '\n' ' '; echo
done
