# k2-leg iteration: the cfg5/stress/sparse parity tests, the bench with the cfg5 k2 leg, sp_level laps. OUT names gpurun_out/<OUT>.
set -u
O=gpurun_out/${OUT:-k2}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q -m gpu --timeout 300 --timeout-method thread -k "cfg5 or stress or synthetic or sparse or decline" > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 400 python bench.py --cpu-sample 0 --e2e= --pcie 0 --k2-contigs 6250 > $O/bench.json 2> $O/bench.err || exit 1
python scripts/show_bench.py $O/bench.json | head -3
WAAFLE_HIP_LIB=waafle_amd/libwaafle_hip_stamps.so timeout -k 10 300 python scripts/wave_stamps.py --config cfg5 --contigs 6250 > $O/stamps_cfg5.json 2> $O/stamps_cfg5.err
