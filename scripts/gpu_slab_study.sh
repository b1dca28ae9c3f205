# Where the 1024 x 8192 slab (config 4's per-GPU shard at N = 8) loses against
# the whole 8192^2 grid: launch time against the
# steps per launch K (t = a + b K separates per-launch from per-step cost), and
# against the launch grid (TFG_BLOCKS), on one box.  JSON lines in
# gpurun_out/slab/study.jsonl.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/slab; mkdir -p $OUT
: > $OUT/study.jsonl
run() {  # tag rows fuse steps [env...]
  local tag=$1 rows=$2 fuse=$3 steps=$4; shift 4
  env "$@" timeout -k 10 300 python bench.py --ny $rows --nx 8192 --fuse $fuse --steps $steps --warmup $fuse \
      --no-cpu-baseline > $OUT/$tag.log 2>&1 || { tail -5 $OUT/$tag.log; exit 1; }
  python3 - "$tag" "$rows" "$fuse" "$*" $OUT/$tag.log >> $OUT/study.jsonl <<'PY'
import json, sys
tag, rows, fuse, env, log = sys.argv[1:6]
r = json.loads([l for l in open(log) if l.startswith("{")][-1])
L = r["launches"]
print(json.dumps({"tag": tag, "rows": int(rows), "fuse": int(fuse), "env": env, "G_cell_updates_s": r["value"] / 1e9,
                  "launch_ms_mean": L["ms_mean"], "launch_ms_min": L["ms_min"], "launch_ms_each": L["ms_each"],
                  "frac": r["roofline"]["frac"]}))
PY
  tail -1 $OUT/study.jsonl | cut -c1-200
}
run full_k96 8192 96 288
for k in 48 96 192 384; do run slab_k$k 1024 $k $((k * 4)); done
for b in 8192 16384 65536; do run slab_k192_b$b 1024 192 768 TFG_BLOCKS=$b; done
run full_k96_again 8192 96 288
