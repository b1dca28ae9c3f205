# Many single-catchment BMI models in one process, NextGen's per-model order
# against the deferred ensemble order (defer_update: one k_cell_many launch per
# step serves every model): per-instance step cost at 1 / 50 / 500 / 2000
# models, and the kernel trace of the 500-model ensemble (device time per
# k_cell_many launch).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-many_batched}; mkdir -p $OUT
for spec in "1 400" "50 40" "500 16" "2000 6"; do
  set -- $spec
  timeout -k 10 300 python tests/diagnostics/bmi_many_instances.py $1 $2 >> $OUT/many.log 2>&1 || { tail -5 $OUT/many.log; exit 1; }
  tail -1 $OUT/many.log
  timeout -k 10 300 python tests/diagnostics/bmi_many_instances.py $1 $2 defer ensemble >> $OUT/many.log 2>&1 || { tail -5 $OUT/many.log; exit 1; }
  tail -1 $OUT/many.log
done
timeout -k 10 300 python tests/diagnostics/bmi_many_instances.py 500 16 defer >> $OUT/many.log 2>&1 || { tail -5 $OUT/many.log; exit 1; }
tail -1 $OUT/many.log
timeout -k 10 300 python tests/diagnostics/bmi_many_instances.py 2000 6 distinct defer ensemble >> $OUT/many.log 2>&1 || { tail -5 $OUT/many.log; exit 1; }
tail -1 $OUT/many.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace500 -o run --output-format csv -- python3 tests/diagnostics/bmi_many_instances.py 500 16 defer ensemble > $OUT/trace500.log 2>&1 || { tail -5 $OUT/trace500.log; exit 1; }
tail -1 $OUT/trace500.log
