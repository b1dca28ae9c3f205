# Same-box A/B of library variants at 8192^2 with the driver's bench command,
# alternating; each entry of VARIANTS is lib[:TFG_BLOCKS] (blocks optional).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-ab_variants}; mkdir -p $OUT
for rep in ${REPS:-1 2}; do
  for v in $VARIANTS; do
    lib=${v%%:*}; blk=${v#*:}; [ "$blk" = "$v" ] && blk=
    if [ -n "$blk" ]; then export TFG_BLOCKS=$blk; else unset TFG_BLOCKS; fi
    TFG_LIB=$PWD/$lib timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/run.log 2>&1 || { echo "$v bench fail"; tail -3 $OUT/run.log; exit 1; }
    python -c "import json; r=json.loads([l for l in open('$OUT/run.log') if l.startswith('{')][-1]); print(json.dumps({'variant': '$v', 'G': round(r['value']/1e9, 2), 'ms_mean': round(r['launches']['ms_mean'], 3)}))" | tee -a $OUT/results.jsonl
  done
done
