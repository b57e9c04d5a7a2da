# Summarise a gpu_iter.sh round: test tail, ms/pass per config, top kernels, per-level trace.
O=gpurun_out/${1:-iter}
tail -1 $O/gpu_tests.log 2>/dev/null
for c in cfg2 cfg3 cfg5; do
  python -c "import json; d=json.load(open('$O/$c.json')); print('$c', round(d['value']), 'contigs/s', round(d['ms_per_step'], 3), 'ms')" 2>/dev/null
done
head -14 $O/prof.txt 2>/dev/null
cat $O/levels.txt 2>/dev/null
