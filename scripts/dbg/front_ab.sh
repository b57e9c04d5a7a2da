set -u
O=gpurun_out/${OUT:-front1}; mkdir -p $O
timeout -k 10 300 env WAAFLE_HIP_LIB=ab_old/libwaafle_hip.so python3 -u scripts/dbg/front_ab.py dump $O/old.npz > $O/old.log 2>&1 || { tail -20 $O/old.log; exit 1; }
cat $O/old.log
timeout -k 10 300 python3 -u scripts/dbg/front_ab.py dump $O/new.npz > $O/new.log 2>&1 || { tail -20 $O/new.log; exit 1; }
cat $O/new.log
python3 scripts/dbg/front_ab.py compare $O/old.npz $O/new.npz
timeout -k 10 300 python3 bench.py --config cfg5 --contigs 6250 --cpu-sample 0 --e2e= --pcie 0 --shares= --k2-contigs 0 --steps 5 --warmup 2 > $O/b5.json 2> $O/b5.err || { tail -20 $O/b5.err; exit 1; }
python3 scripts/show_bench.py $O/b5.json
