# HBM traffic of the ice-flow kernels (FETCH_SIZE / WRITE_SIZE in separate passes)
# on tests/diagnostics/ice_flow_timing.py at 8192^2.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc_flow}
mkdir -p $OUT
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/p$i -o run -- python3 tests/diagnostics/ice_flow_timing.py 8192 8192 5 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($c) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
for k in "k_ice_flow<float, false>" "k_ice_flow<float, true>" "k_flow_commit"; do
  echo "== $k"; python3 scripts/pmc_summary.py $OUT "$k"
done
