# Workgroup count (TFG_BLOCKS) against the default (128 per CU = 32768) with the
# driver's bench command at 8192^2 and on the N = 8 shard (1024 x 8192),
# alternating on one box; stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-blocks_driver}; mkdir -p $OUT
for rep in ${REPS:-1 2}; do
  for b in ${BLOCKS:-16384 32768 65536}; do
    for shape in ${SHAPES:-"8192 8192" "1024 8192"}; do
      set -- $shape
      TFG_BLOCKS=$b timeout -k 10 300 python bench.py --ny $1 --nx $2 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/run.log 2>&1 || { echo "blocks $b $shape fail"; tail -3 $OUT/run.log; exit 1; }
      python -c "import json; r=json.loads([l for l in open('$OUT/run.log') if l.startswith('{')][-1]); l=r['launches']; print(json.dumps({'blocks': $b, 'shape': '$1x$2', 'G': round(r['value']/1e9, 2), 'K': l['steps_each'], 'ms_mean': round(l['ms_mean'], 3)}))" | tee -a $OUT/results.jsonl
    done
  done
done
