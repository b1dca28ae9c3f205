# Round 5: the in-tree library's deep-launch tails (gpu_r5_tail.sh, SAMPLES), a same-box A/B against
# variant builds (gpu_r5_ab.sh, ABLIBS), then the GPU suite (gpu_tests.sh) unless NO_SUITE is set.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
main=topoflow-glacier_amd/topoflow_glacier/_tfg.so
LIB=$main TAG=${TAG:-r5chk} SAMPLES="${SAMPLES:-n4 n2 n8 cfg3 cfg5}" bash scripts/gpu_r5_tail.sh || exit $?
if [ -n "$ABLIBS" ]; then
  LIBS="$main $ABLIBS" TAG=${TAG:-r5chk}_ab REPS=${REPS:-2} bash scripts/gpu_r5_ab.sh || exit $?
fi
[ -n "$NO_SUITE" ] || bash scripts/gpu_tests.sh
