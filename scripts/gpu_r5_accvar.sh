# Round 5: accuracy variants of the fp32 turbulent terms (diag_libs, LIBS): a same-box speed A/B against the
# in-tree library, then each variant's parity samples at the ranks with the largest round-5 errors (RANKS).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5acc}_ab REPS=1 LIBS="topoflow-glacier_amd/topoflow_glacier/_tfg.so $LIBS" bash scripts/gpu_r5_ab.sh || exit $?
for lib in $LIBS; do
  v=$(basename $lib .so)
  LIB=$lib TAG=${TAG:-r5acc}_$v RANKS="${RANKS:-4:2 8:5 4:3 8:7}" bash scripts/gpu_r5_ranks.sh || exit $?
done
# F64LIBS: a same-box A/B of fp64 variants against the in-tree library at 4096^2 (REPS64 rounds)
[ -z "$F64LIBS" ] || TAG=${TAG:-r5acc}_ab64 REPS=${REPS64:-2} BENCH_ARGS="--engine float64 --ny 4096 --nx 4096" \
  LIBS="topoflow-glacier_amd/topoflow_glacier/_tfg.so $F64LIBS" bash scripts/gpu_r5_ab.sh
