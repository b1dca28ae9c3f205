# Does the launch time keep falling with the time spent warming up?  The
# per-launch times of the driver's command drift down ~2 % over its 12 timed
# launches (profiles/r3i_bench_driver.json).  Whole grid (96-step launches) and
# the 1024 x 8192 slab (192-step launches) after warm-ups of one launch, ~0.5 s
# and ~2 s of launches; same box.  JSON lines in gpurun_out/warmup_time/study.jsonl.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/warmup_time; mkdir -p $OUT
: > $OUT/study.jsonl
run() {  # tag rows warmup_steps
  local tag=$1 rows=$2 warm=$3
  timeout -k 10 300 python bench.py --ny $rows --nx 8192 --steps 20 --warmup $warm --no-cpu-baseline > $OUT/$tag.log 2>&1 || { tail -5 $OUT/$tag.log; exit 1; }
  python3 - "$tag" "$rows" "$warm" $OUT/$tag.log >> $OUT/study.jsonl <<'PY'
import json, sys
tag, rows, warm, log = sys.argv[1:5]
r = json.loads([l for l in open(log) if l.startswith("{")][-1])
print(json.dumps({"tag": tag, "rows": int(rows), "warmup_steps": int(warm), "G_cell_updates_s": r["value"] / 1e9,
                  "launch_ms_each": r["launches"]["ms_each"]}))
PY
  tail -1 $OUT/study.jsonl | cut -c1-250
}
for pass in a b; do
  run ${pass}_full_w96 8192 96 || exit 1
  run ${pass}_full_w960 8192 960 || exit 1
  run ${pass}_full_w3840 8192 3840 || exit 1
  run ${pass}_slab_w192 1024 192 || exit 1
  run ${pass}_slab_w7680 1024 7680 || exit 1
  run ${pass}_slab_w23040 1024 23040 || exit 1
done
