# Same-box A/B of library variants (abvar/*.so through TFG_LIB), alternating:
# the driver's bench command at 8192^2 (automatic depth), config 5's slab
# (43 catchments, dt = 0.25 h) and config 2's 1024^2; stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-ab_driver}; mkdir -p $OUT
one() { lib=$1; shift; name=$1; shift
  TFG_LIB=$PWD/$lib timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > $OUT/run.log 2>&1 || { echo "$lib $name bench fail"; tail -3 $OUT/run.log; return 1; }
  python -c "import json; r=json.loads([l for l in open('$OUT/run.log') if l.startswith('{')][-1]); l=r['launches']; print(json.dumps({'lib': '$lib', 'case': '$name', 'G': round(r['value']/1e9, 2), 'frac': round(r['roofline']['frac'], 4), 'K': l['steps_each'], 'ms_mean': round(l['ms_mean'], 3), 'ms_min': round(l['ms_min'], 3)}))" | tee -a $OUT/results.jsonl
}
for rep in ${REPS:-1 2 3}; do
  for lib in ${AB_LIBS:-abvar/*.so}; do
    one $lib driver_8192sq --gpus 1 --steps 20 --warmup 5 || exit 1
    one $lib cfg5_slab --ny 2048 --nx 16384 --dt 0.25 --catchments 43 --steps 480 || exit 1
    one $lib cfg2_1024sq --ny 1024 --nx 1024 --fuse 120 --steps 3840 --warmup 2400 || exit 1
  done
done
