# Round 5: parity tails (tests/diagnostics/parity_tail.py) of several library variants (LIBS) on SAMPLES.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for lib in ${LIBS}; do
  v=$(basename $lib .so)
  LIB=$lib TAG=${TAG:-r5tab}_$v SAMPLES="${SAMPLES:-n4 n2 cfg4 cfg5}" bash scripts/gpu_r5_tail.sh || exit $?
done
