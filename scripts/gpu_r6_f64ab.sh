# Round 6: fp64-engine variants (diag_libs builds, LIBS): same-box A/B of the fp64 bench at 4096^2
# (192-step launches), alternating, REPS rounds, then one PMC pass per variant (SQ_INSTS_VALU per wave and
# cell-step of the timed kernel; scripts/issue_summary.py's arithmetic) and optionally F32=1 the fp32 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${TAG:-r6f64ab}
mkdir -p gpurun_out/$tag
ARGS="--engine float64 --ny 4096 --nx 4096 --fuse 192 --steps 384 --warmup 192"
RUNS=""
for l in $LIBS; do RUNS="$RUNS $l|${ARGS// /,}"; [ -n "$F32" ] && RUNS="$RUNS $l|--fuse,128"; done
TAG=$tag/ab RUNS="$RUNS" REPS=${REPS:-2} bash scripts/gpu_r6_ab.sh || exit $?
for l in $LIBS; do
  v=$(basename $l .so)
  TFG_LIB=$PWD/$l timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES --output-format csv \
    -d gpurun_out/$tag/pmc_$v -o run -- python3 bench.py $ARGS --steps 192 --warmup 192 --no-cpu-baseline --no-parity \
    --no-dropin > gpurun_out/$tag/pmc_$v.log 2>&1
  rc=$?; echo "pmc $v rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/$tag/pmc_$v.log; exit $rc; }
  python3 - gpurun_out/$tag/pmc_$v <<'EOF'
import csv, glob, sys
from collections import defaultdict
per = defaultdict(lambda: defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_fused<double, true, false, false, false, 1, false, false>" in r["Kernel_Name"]:
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
d = [v for v in per.values() if v.get("SQ_WAVES")]
top = max(x["SQ_INSTS_VALU"] for x in d)
d = [x for x in d if x["SQ_INSTS_VALU"] > 0.5 * top]  # whole 192-step launches (not the bench's lead-in)
ws = 4096 * 4096 / 64 * 192  # wave-steps of one 192-step launch
m = {c: sum(x[c] for x in d) / len(d) / ws for c in d[0] if c != "SQ_WAVES"}
print(sys.argv[1].split("/")[-1], len(d), "dispatches", {k: round(v, 1) for k, v in m.items()}, flush=True)
EOF
done
