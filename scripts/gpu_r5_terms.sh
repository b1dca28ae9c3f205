# Round 5: accumulated energy-term error of diagnostic builds (tests/diagnostics/term_bias.py),
# LIBS="diag_libs/_tfg_terms_<v>.so ..."; then optional GPU tests (TESTS="pytest node ids").
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-r5terms}
stop() { rc=$1; case $rc in 124|134|137|139) echo "GPU step ended with $rc: stopping"; exit $rc;; esac; }
for lib in ${LIBS}; do
  v=$(basename $lib .so)
  TFG_LIB=$PWD/$lib timeout -k 10 300 python -u tests/diagnostics/term_bias.py gpurun_out/${tag}_$v.json ${ROWS:-2} ${STEPS:-385} \
    > gpurun_out/${tag}_$v.log 2>&1; rc=$?; echo "== $v rc=$rc"; cat gpurun_out/${tag}_$v.log | tail -6; stop $rc; [ $rc -eq 0 ] || exit $rc
done
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTS > gpurun_out/${tag}_tests.log 2>&1
  rc=$?; tail -15 gpurun_out/${tag}_tests.log; exit $rc
fi
