# results of library variant A against the in-tree library on the cfg5 share (front_ab.py)
set -u
O=gpurun_out/${OUT:-fcmp}; mkdir -p $O
timeout -k 10 300 env WAAFLE_HIP_LIB=waafle_amd/libwaafle_hip_$A.so python3 -u scripts/dbg/front_ab.py dump $O/a.npz > $O/a.log 2>&1 || { tail -20 $O/a.log; exit 1; }
timeout -k 10 300 python3 -u scripts/dbg/front_ab.py dump $O/main.npz > $O/main.log 2>&1 || { tail -20 $O/main.log; exit 1; }
cat $O/a.log $O/main.log
python3 scripts/dbg/front_ab.py compare $O/a.npz $O/main.npz
