# round-3 GPU session: parity tests, smoke, the default bench line (cfg4 + the cfg5 k2 leg +
# CPU legs + scopes ii/iii), kernel-trace stats of cfg4 and of the cfg5 6,250-contig share.
# OUT names gpurun_out/<OUT>.  TESTS: pytest targets (SKIP_TESTS=1: none); BENCH=0 skips the
# default bench (BENCH_ARGS adds to it); PROF=0 skips the profiles; AB="name=args;..." adds
# bench runs with those arguments (QUICK args: no CPU legs); VARIANTS="skip8 ..." times the
# diagnostic builds waafle_amd/libwaafle_hip_<v>.so on cfg4.
set -u
O=gpurun_out/${OUT:-r3}; mkdir -p $O
export TMPDIR=/tmp
QUICK="--cpu-sample 0 --e2e= --pcie 0"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 1500 python -u -m pytest ${TESTS:-tests} -x -q -m gpu --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || exit $?
fi
if [ -n "${AB:-}" ]; then
  IFS=';' read -ra runs <<< "$AB"
  for r in "${runs[@]}"; do
    name=${r%%=*}; args=${r#*=}
    timeout -k 10 600 python bench.py $QUICK $args > $O/ab_$name.json 2> $O/ab_$name.err || exit $?
  done
fi
for v in ${VARIANTS:-}; do
  WAAFLE_HIP_LIB=waafle_amd/libwaafle_hip_$v.so timeout -k 10 600 python bench.py $QUICK --k2-contigs 0 --steps 5 > $O/var_$v.json 2> $O/var_$v.err || exit $?
done
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof5 -o run --output-format csv -- python3 bench.py --config cfg5 --contigs 6250 --k2-contigs 0 $QUICK --steps 4 --warmup 1 ${PROF_ARGS:-} > $O/prof5.json 2> $O/prof5.err || exit $?
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof4 -o run --output-format csv -- python3 bench.py --k2-contigs 0 $QUICK --steps 4 --warmup 1 ${PROF_ARGS:-} > $O/prof4.json 2> $O/prof4.err || exit $?
fi
echo done
