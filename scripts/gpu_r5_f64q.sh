# Round 5, fp64 engine: same-box A/B of the in-tree library against the session-start build and the
# Halley-root build (gpu_r5_ab.sh at 4096^2), then the final-code record (gpu_r5_final_c.sh: GPU suite,
# fp64 PMC profile, bench line, issue counters of both engines, smoke).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
LIBS="diag_libs/_tfg_base.so diag_libs/_tfg_h10.so topoflow-glacier_amd/topoflow_glacier/_tfg.so" TAG=${TAG:-r5q}_ab \
  REPS=2 BENCH_ARGS="--engine float64 --ny 4096 --nx 4096" bash scripts/gpu_r5_ab.sh || exit $?
TAG=${TAG:-r5q} bash scripts/gpu_r5_final_c.sh
