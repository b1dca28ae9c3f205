# Same-box A/B of the fp64 engine with em_air's (e/T)^(1/7) as exp(log(x)/7)
# (abvar/b_root7.so) against the general pow (abvar/a_base.so): 4096^2 bulk
# rate and single-catchment BMI latency (gpu_ab_exact.sh), k_cell_run step cost
# (gpu_ab_cellrun.sh); then the GPU suite on the in-tree build, with reports.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-ab_root7}; mkdir -p $OUT
for rep in 1 2; do AB_LIBS="abvar/a_base.so abvar/b_root7.so" bash scripts/gpu_ab_exact.sh || exit 1; done 2>&1 | tee $OUT/ab_exact.log
AB_LIBS="abvar/a_base.so abvar/b_root7.so" TAG=${TAG:-ab_root7}/cellrun bash scripts/gpu_ab_cellrun.sh 2>&1 | tee $OUT/ab_cellrun.log || exit 1
TFG_REPORT_DIR=$OUT/reports timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1; rc=$?; tail -2 $OUT/gpu_tests.log; exit $rc
