# Per-launch times of the strong-scaling slabs (8192/N rows x 8192) as the
# driver runs them (--steps 20: three 192-step launches), after a short
# (--warmup 5, the driver's) and a one-launch (--warmup 192) warm-up.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-slab_warmup}; mkdir -p $OUT
for rows in ${ROWS:-4096 2048 1024}; do
  for w in 5 192; do
    timeout -k 10 300 python bench.py --ny $rows --nx 8192 --steps 20 --warmup $w --no-cpu-baseline --no-pcie > $OUT/r${rows}_w$w.log 2>&1 || { tail -5 $OUT/r${rows}_w$w.log; exit 1; }
    grep '^{' $OUT/r${rows}_w$w.log | tail -1 > $OUT/r${rows}_w$w.json
    python3 -c "import json; r=json.load(open('$OUT/r${rows}_w$w.json')); print('$rows rows warmup $w', '%.2f G/s'%(r['value']/1e9), r['launches']['ms_each'])"
  done
done
