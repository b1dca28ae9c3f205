# PMC passes on the bench workload (one counter set per pass; no tracing domains),
# then the 4-byte-lane calibration passes on tools/hbm_mix, then the profile JSON
# bench.py quotes (scripts/pmc_profile.py; PMC_PROFILE names it).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${PMC_TAG:-pmc}
mkdir -p $OUT
# every k_fused dispatch of this run is a full 128-step launch (warm-up included;
# no parity or drop-in legs, whose launches would enter the per-dispatch means)
ARGS="${PMC_ARGS:---ny 8192 --nx 8192 --fuse 128 --steps 768 --warmup 128 --no-cpu-baseline --no-dropin --no-parity}"
i=0
while IFS= read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $line --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($line) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done <<PASSES
FETCH_SIZE
WRITE_SIZE
${PMC_EXTRA:-}
PASSES
for c in FETCH_SIZE WRITE_SIZE; do
  d=$OUT/cal_$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d $d -o run -- tools/hbm_mix 67108864 8 2048 0 cal > $d.log 2>&1
  rc=$?; echo "calibration $c rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $d.log; exit $rc; fi
done
python3 scripts/pmc_profile.py $OUT ${PMC_PROFILE:-$OUT/profile.json} ${PMC_SHAPE:-8192 8192 128} 67108864 8 ${PMC_ENGINE:-float32}
