# Same-box A/B of library variants on the one-cell multi-step kernel
# (k_cell_run: update_until / bulk runs of one catchment): device time of 1-,
# 2-, 4- and 8-step launches under rocprofv3 (tests/diagnostics/one_cell_step_cost.py),
# alternating A B A B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab_cellrun}; mkdir -p $OUT
i=0
for rep in 1 2; do
  for lib in ${AB_LIBS:-abvar2/*.so}; do
    i=$((i+1))
    TFG_LIB=$PWD/$lib timeout -k 10 180 rocprofv3 --kernel-trace -d $OUT/t$i -o run --output-format csv -- python3 tests/diagnostics/one_cell_step_cost.py > $OUT/t$i.log 2>&1 || { echo "$lib fail"; tail -5 $OUT/t$i.log; exit 1; }
    echo "$lib $(python3 tests/diagnostics/one_cell_step_cost.py --summary $OUT/t$i | tail -1)"
  done
done
