# Launch depth on the small BASELINE grids after a long warm-up (config 2's
# 1024^2 and 2048^2): is there a per-launch cost that deeper launches amortise,
# once the slow first launches of a fresh process (clock ramp) are excluded?
# Alternates the depths twice on one box; stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-small_depth}; mkdir -p $OUT
for rep in 1 2; do
  for g in ${GRIDS:-1024 2048}; do
    if [ $g -le 1024 ]; then KL="${KS:-120 480 1920 3840}"; else KL="${KS2:-96 384 1536}"; fi
    for k in $KL; do
      timeout -k 10 300 python bench.py --ny $g --nx $g --fuse $k --steps ${STEPS:-15360} --warmup ${WARM:-24000} --no-cpu-baseline > $OUT/run.log 2>&1 || { echo "$g K=$k bench fail"; tail -3 $OUT/run.log; exit 1; }
      python -c "import json; r=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); l=r['launches']; print(json.dumps({'grid': $g, 'K': $k, 'G': round(r['value']/1e9, 2), 'frac': round(r['roofline']['frac'], 4), 'ms_mean': round(l['ms_mean'], 4), 'ms_min': round(l['ms_min'], 4), 'ms_max': round(l['ms_max'], 4), 'launches': l['count']}))" | tee -a $OUT/results.jsonl
    done
  done
done
