# Round 5: the fp32 engine's forcing prefetch through an LDS ring (global_load_lds_dword, three steps ahead)
# against the in-tree library: same-box A/B at the default bench workload (8192^2, 128-step launches), then
# the GPU suite against the variant (TFG_LIB).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5lds}
mkdir -p gpurun_out/$TAG
LIBS="topoflow-glacier_amd/topoflow_glacier/_tfg.so diag_libs/_tfg_lds.so" TAG=${TAG}_ab REPS=${REPS:-3} \
  bash scripts/gpu_r5_ab.sh || exit $?
TFG_LIB=$PWD/diag_libs/_tfg_lds.so timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/$TAG/gpu_tests.log | tail -8; exit $rc
