# Round 5: the wet bulb's arctangent from its two operands (atan_q) and square root (sqrt_k), with and
# without exp of degree 9 / root7 by one Newton or Halley step (LIBS, PARITY_LIBS, FASTMATH_LIBS): fp64 engine A/B at 4096^2 (gpu_r5_ab.sh), then the
# fp64 parity tests that the changes touch, run against each variant library (TFG_LIB).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
LIBS="${LIBS:-diag_libs/_tfg_base.so diag_libs/_tfg_wb.so diag_libs/_tfg_wb2.so}" TAG=${TAG:-r5wb} REPS=${REPS:-2} \
  BENCH_ARGS="--engine float64 --ny 4096 --nx 4096" bash scripts/gpu_r5_ab.sh || exit $?
for v in ${PARITY_LIBS:-_tfg_wb _tfg_wb2}; do
  k="fp64 or one_cell or satterlund or power_rewrites"
  [ -n "$FASTMATH_LIBS" ] && [[ " $FASTMATH_LIBS " == *" $v "* ]] && k="$k or fastmath"  # the host build's exp
  TFG_LIB=$PWD/diag_libs/$v.so TFG_REPORT_DIR=gpurun_out/${TAG:-r5wb}_$v timeout -k 10 600 python -u -m pytest -x -q \
    --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_power_rewrites.py tests/test_fastmath.py \
    -m gpu -k "$k" > gpurun_out/${TAG:-r5wb}_parity_$v.log 2>&1
  rc=$?; echo "$v parity rc=$rc"; tail -3 gpurun_out/${TAG:-r5wb}_parity_$v.log; [ $rc -eq 0 ] || { [ -n "$KEEP_GOING" ] && [ $rc -eq 1 ]; } || exit $rc  # go on only after plain test failures
done
