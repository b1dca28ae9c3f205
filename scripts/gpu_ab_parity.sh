# Same-box A/B of library variants (abvar/*.so) with the driver's bench command
# including its CPU legs, so each line carries the sample parity against the
# oracle (pure-relative miss fractions, melt-out flips) beside the rate.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-ab_parity}; mkdir -p $OUT
# the CPU legs print nothing for minutes: a heartbeat file keeps gpurun's silence watchdog informed
( while sleep 30; do date +%s >> $OUT/heartbeat.log; done ) & HB=$!
trap "kill $HB" EXIT
for rep in ${REPS:-1 2}; do
  for lib in ${AB_LIBS:-abvar/*.so}; do
    t0=$(date +%s)
    TFG_LIB=$PWD/$lib timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-cells ${CPU_CELLS:-65536} --cpu-steps 96 > $OUT/run.log 2>&1 || { echo "$lib fail rc=$? after $(( $(date +%s) - t0 )) s"; tail -3 $OUT/run.log; exit 1; }
    echo "$lib bench took $(( $(date +%s) - t0 )) s"
    python -c "
import json; r=json.loads([l for l in open('$OUT/run.log') if l.startswith('{')][-1]); sp=r['sample_parity']
print(json.dumps({'lib': '$lib', 'G': round(r['value']/1e9, 2), 'max_floored_rel': sp['max_floored_rel'], 'flips': sp['melt_out_flips'], 'flip_ratio': round(sp['flip_ratio'], 3), 'pure_rel': {k: round(v, 6) for k, v in sp['frac_above_pure_rel_1e-5'].items()}, 'ok': sp['ok']}))" | tee -a $OUT/results.jsonl
  done
done
