# The 1024 x 8192 slab (config 4's per-GPU shard at N = 8): does its deficit
# against the whole grid come from the GPU's clock ramp (a warm-up measured in
# time rather than in launches) or from the power-of-two plane stride
# (n_pad = 2^23 cells: every plane of a step at the same channel offset)?
# Launch depth 96/192/384, warm-up one launch vs ten launches, plane skew
# 0/256/4096 cells (TFG_PLANE_SKEW).  JSON lines in gpurun_out/slab_skew/study.jsonl.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/slab_skew; mkdir -p $OUT
: > $OUT/study.jsonl
run() {  # tag rows fuse steps warmup skew
  local tag=$1 rows=$2 fuse=$3 steps=$4 warm=$5 sk=$6
  TFG_PLANE_SKEW=$sk timeout -k 10 300 python bench.py --ny $rows --nx 8192 --fuse $fuse --steps $steps --warmup $warm \
      --no-cpu-baseline > $OUT/$tag.log 2>&1 || { tail -5 $OUT/$tag.log; exit 1; }
  python3 - "$tag" "$rows" "$fuse" "$warm" "$sk" $OUT/$tag.log >> $OUT/study.jsonl <<'PY'
import json, sys
tag, rows, fuse, warm, sk, log = sys.argv[1:7]
r = json.loads([l for l in open(log) if l.startswith("{")][-1])
L = r["launches"]
cells = int(rows) * 8192
print(json.dumps({"tag": tag, "rows": int(rows), "fuse": int(fuse), "warmup": int(warm), "skew": int(sk),
                  "G_cell_updates_s": r["value"] / 1e9, "G_at_min_launch": cells * int(fuse) / L["ms_min"] / 1e6,
                  "launch_ms_each": L["ms_each"]}))
PY
  tail -1 $OUT/study.jsonl | cut -c1-220
}
for sk in 0 256 4096; do
  for k in 96 192 384; do
    run s${sk}_k${k}_w1 1024 $k $((k * 4)) $k $sk || exit 1
    run s${sk}_k${k}_w10 1024 $k $((k * 4)) $((k * 10)) $sk || exit 1
  done
done
for sk in 0 256; do run full_s${sk} 8192 96 288 96 $sk || exit 1; done
