# Launch depth on the shards of 2^24 cells and fewer (the N = 4 and N = 8
# strong-scaling shards of config 4, and 2048^2), driver-like warm-up, 4608
# timed steps (at least 6 launches), alternating the depths twice on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-depth_shapes}; mkdir -p $OUT
run() { ny=$1; nx=$2; k=$3
  timeout -k 10 300 python bench.py --ny $ny --nx $nx --fuse $k --steps ${STEPS:-4608} --warmup 5 --no-cpu-baseline > $OUT/run.log 2>&1 || { echo "${ny}x$nx K=$k bench fail"; tail -3 $OUT/run.log; return 1; }
  python -c "import json; r=json.loads([l for l in open('$OUT/run.log') if l.startswith('{')][-1]); l=r['launches']; print(json.dumps({'shape': '${ny}x$nx', 'K': $k, 'G': round(r['value']/1e9, 2), 'frac': round(r['roofline']['frac'], 4), 'ms_first': round(l['ms_each'][0], 3), 'ms_mean': round(l['ms_mean'], 3), 'ms_min': round(l['ms_min'], 3), 'launches': l['count']}))" | tee -a $OUT/results.jsonl
}
for rep in 1 2; do
  for k in ${K8:-384 768 1024}; do run 1024 8192 $k || exit 1; done
  for k in ${K4:-384 512}; do run 2048 8192 $k || exit 1; done
  for k in ${K2:-384 768 1536}; do run 2048 2048 $k || exit 1; done
done
