# fp32 engine accuracy variants (TFG_ACC, csrc/tfg_physics.hpp) against the
# default build, same box, alternating: bench.py's throughput and its parity
# check (pure-relative misses, max floored error) per build.  Libraries:
# diag_libs/_tfg_acc<N>.so built with -DTFG_ACC=<N> (scripts/build_variants below).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-r4b}
i=0
for v in ${VARIANTS:-base acc1 acc7 acc23 base acc15 acc31 base}; do
  i=$((i+1))
  lib=topoflow-glacier_amd/topoflow_glacier/_tfg.so
  [ "$v" = base ] || lib=diag_libs/_tfg_$v.so
  TFG_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-dropin ${BENCH_ARGS:-} \
      > gpurun_out/${tag}_${i}_${v}.json 2> gpurun_out/${tag}_${i}_${v}.err
  rc=$?
  python - "$v" gpurun_out/${tag}_${i}_${v}.json <<'PY'
import json, sys
try:
    d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
    sp = d["sample_parity"]
    print(sys.argv[1], f"{d['value']/1e9:.2f} G", f"frac {d['roofline']['frac']:.4f}", f"err {sp['max_floored_rel']:.2e}",
          "pure%", {k: round(v * 100, 4) for k, v in sp["frac_above_pure_rel_1e-5"].items()},
          "flips", sp["melt_out_flips"], "/", sp["flips_fp64_baseline"], "ok", sp["ok"], flush=True)
except Exception as e:
    print(sys.argv[1], "no result", e)
PY
  case $rc in 0) ;; 124|134|137|139) echo "GPU step ended with $rc: stopping"; exit $rc;; *) exit $rc;; esac
done
