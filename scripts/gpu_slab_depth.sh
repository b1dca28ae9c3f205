# Launch depth for the strong-scaling slabs as the driver would time them
# (--warmup 5, 1152 timed steps): 4096 rows at K = 192; 2048 and 1024 rows at
# K = 192 and 384; the whole grid at K = 96.  Two passes (same box) so that
# the spread between processes shows.  JSON lines in gpurun_out/slab_depth/study.jsonl.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/slab_depth; mkdir -p $OUT
: > $OUT/study.jsonl
run() {  # tag rows fuse
  local tag=$1 rows=$2 fuse=$3
  timeout -k 10 300 python bench.py --ny $rows --nx 8192 --fuse $fuse --steps 1152 --warmup 5 \
      --no-cpu-baseline > $OUT/$tag.log 2>&1 || { tail -5 $OUT/$tag.log; exit 1; }
  python3 - "$tag" "$rows" "$fuse" $OUT/$tag.log >> $OUT/study.jsonl <<'PY'
import json, sys
tag, rows, fuse, log = sys.argv[1:5]
r = json.loads([l for l in open(log) if l.startswith("{")][-1])
L = r["launches"]
print(json.dumps({"tag": tag, "rows": int(rows), "fuse": int(fuse), "G_cell_updates_s": r["value"] / 1e9,
                  "G_at_min_launch": int(rows) * 8192 * int(fuse) / L["ms_min"] / 1e6, "launch_ms_each": L["ms_each"]}))
PY
  tail -1 $OUT/study.jsonl | cut -c1-220
}
for pass in a b; do
  run ${pass}_r4096_k192 4096 192 || exit 1
  for rows in 2048 1024; do
    for k in 192 384; do run ${pass}_r${rows}_k$k $rows $k || exit 1; done
  done
  run ${pass}_r8192_k96 8192 96 || exit 1
done
