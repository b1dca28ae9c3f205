# The optional lateral conduction term at 8192^2: timing (tests/diagnostics/
# conduction_timing.py), rocprofv3 kernel stats, and HBM traffic of
# k_conduction (FETCH_SIZE / WRITE_SIZE in separate passes).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-cond}
mkdir -p $OUT
timeout -k 10 300 python3 tests/diagnostics/conduction_timing.py 8192 8192 20 96 > $OUT/timing.log 2>&1
rc=$?; echo "timing rc=$rc"; tail -1 $OUT/timing.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tests/diagnostics/conduction_timing.py 8192 8192 20 96 > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/p$i -o run -- python3 tests/diagnostics/conduction_timing.py 8192 8192 5 96 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($c) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
python3 scripts/pmc_summary.py $OUT "k_conduction<float>"
