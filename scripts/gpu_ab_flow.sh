# Same-box A/B of ice-flow kernel variants (abvar/*.so), alternating A B C ...:
# tests/diagnostics/ice_flow_timing.py at 8192^2; stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abflow
for rep in 1 2; do
  for lib in ${AB_LIBS:-abvar/*.so}; do
    TFG_LIB=$PWD/$lib timeout -k 10 120 python -u tests/diagnostics/ice_flow_timing.py 8192 8192 100 > gpurun_out/abflow/run.log 2>&1 || { echo "$lib fail"; tail -3 gpurun_out/abflow/run.log; exit 1; }
    echo "$lib $(tail -1 gpurun_out/abflow/run.log)"
  done
done
