# NextGen's many-instance pattern: per-instance step cost at 1 / 50 / 500 / 2000
# one-cell BMI instances, and the kernel trace of the 500-instance run (device
# time per k_fused launch vs the host-side cost).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-many}; mkdir -p $OUT
[ -n "$SPLIT_ONLY" ] || for spec in "1 400" "50 40" "500 16" "2000 6"; do
  set -- $spec
  timeout -k 10 300 python tests/diagnostics/bmi_many_instances.py $1 $2 >> $OUT/many.log 2>&1 || { tail -5 $OUT/many.log; exit 1; }
  tail -1 $OUT/many.log
done
[ -n "$SPLIT_ONLY" ] || timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace500 -o run --output-format csv -- python3 tests/diagnostics/bmi_many_instances.py 500 8 > $OUT/trace500.log 2>&1 || { tail -5 $OUT/trace500.log; exit 1; }
[ -n "$SPLIT_ONLY" ] || tail -1 $OUT/trace500.log
[ -n "$SPLIT_ONLY" ] || timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace1 -o run --output-format csv -- python3 tests/diagnostics/bmi_many_instances.py 1 400 > $OUT/trace1.log 2>&1 || { tail -5 $OUT/trace1.log; exit 1; }
[ -n "$SPLIT_ONLY" ] || tail -1 $OUT/trace1.log
# the diagnostic build splits tfg_update's time (tools/_tfg_timing.so: hipcc ... -DTFG_UPDATE_TIMING)
for spec in "1 400" "500 16" "2000 6" "500 16 distinct" "2000 6 distinct"; do
  set -- $spec
  TFG_LIB=$PWD/tools/_tfg_timing.so timeout -k 10 300 python tests/diagnostics/bmi_many_instances.py $1 $2 $3 >> $OUT/split.log 2>&1 || { tail -5 $OUT/split.log; exit 1; }
  tail -1 $OUT/split.log
done
