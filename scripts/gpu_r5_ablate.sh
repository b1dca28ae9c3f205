# Round 5: cost of the step's parts by ablation (diag_libs builds made by patching a copy of the
# sources; timing only, their results are wrong by construction).  fp64 engine at 4096^2 (F64LIBS),
# then the fp32 kernel's memory-only ceiling at 8192^2 (F32LIBS: the same loads and stores, no physics).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
main=topoflow-glacier_amd/topoflow_glacier/_tfg.so
[ -z "$F64LIBS" ] || TAG=${TAG:-r5abl}64 REPS=${REPS:-1} BENCH_ARGS="--engine float64 --ny 4096 --nx 4096" \
  LIBS="$main $F64LIBS" bash scripts/gpu_r5_ab.sh || exit $?
[ -z "$F32LIBS" ] || TAG=${TAG:-r5abl}32 REPS=${REPS:-1} LIBS="$main $F32LIBS" bash scripts/gpu_r5_ab.sh || exit $?
