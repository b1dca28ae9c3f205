# Strong scaling of BASELINE config 4 (8192^2 partitioned over N GPUs) predicted from
# one GPU: each run is the per-rank slab of the N-GPU partition (8192/N rows x 8192).
# No data-path collective exists, so the N-GPU rate is N x the slab rate minus launch skew.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/strong; mkdir -p $OUT
for rows in 8192 4096 2048 1024; do
  timeout -k 10 300 python bench.py --ny $rows --nx 8192 --steps 480 --no-cpu-baseline --no-pcie > $OUT/rows_$rows.log 2>&1 || { tail -5 $OUT/rows_$rows.log; exit 1; }
  grep '^{' $OUT/rows_$rows.log | tail -1 > $OUT/rows_$rows.json
  python3 -c "import json; r=json.load(open('$OUT/rows_$rows.json')); print('$rows rows', '%.2f G/s'%(r['value']/1e9), 'frac %.3f'%r['roofline']['frac'], 'ms/step %.4f'%r['ms_per_step'])"
done
