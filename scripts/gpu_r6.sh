# Round-6 GPU session helper (one gpurun call; every GPU step under its own time limit).
#   TESTS=1        the GPU suite (TESTSEL narrows it, e.g. "tests/test_gpu_parity.py")
#   SMOKE=1        __graft_entry__.smoke()
#   AB="r5 prod"   same-box A/B of library variants (prod = waafle_amd/libwaafle_hip.so),
#                  REPS times each, bench.py $BENCH_ARGS without the CPU legs
# OUT names gpurun_out/<OUT>.
set -u
O=gpurun_out/${OUT:-r6}; mkdir -p $O
export TMPDIR=/tmp
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TESTSEL:-tests} -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -3 $O/gpu_tests.log
fi
if [ "${SMOKE:-0}" = 1 ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if [ -n "${AB:-}" ]; then
  Q="--cpu-sample 0 --e2e= --pcie 0 --k2-contigs 0 --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS:-}"
  for rep in $(seq 1 ${REPS:-2}); do
    for v in $AB; do
      if [ "$v" = prod ]; then lib=waafle_amd/libwaafle_hip.so; else lib=waafle_amd/libwaafle_hip_$v.so; fi
      WAAFLE_HIP_LIB=$lib timeout -k 10 300 python3 bench.py $Q > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { tail -5 $O/${v}_$rep.err; exit 1; }
      echo "$v rep $rep: $(python3 scripts/show_bench.py $O/${v}_$rep.json | tr '\n' ' ')"
    done
  done
fi
echo r6-done
