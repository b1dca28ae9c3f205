# Same-box A/B of library variants (abvar/*.so) on the optional conduction
# kernel at 8192^2 (tests/diagnostics/conduction_timing.py), alternating, then
# rocprofv3 kernel stats of k_conduction per variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab_cond}; mkdir -p $OUT
for rep in ${REPS:-1 2 3}; do
  for lib in ${AB_LIBS:-abvar/*.so}; do
    TFG_LIB=$PWD/$lib timeout -k 10 300 python tests/diagnostics/conduction_timing.py 8192 8192 20 96 > $OUT/run.log 2>&1 || { echo "$lib fail"; tail -3 $OUT/run.log; exit 1; }
    python -c "import json; r=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print(json.dumps({'lib': '$lib', 'conduction_ms': round(r['conduction_ms'], 4), 'GBps': round(r['GBps'], 1)}))" | tee -a $OUT/results.jsonl
  done
done
for lib in ${AB_LIBS:-abvar/*.so}; do
  n=$(basename $lib .so)
  TFG_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$n -o run --output-format csv -- python3 tests/diagnostics/conduction_timing.py 8192 8192 20 96 > $OUT/trace_$n.log 2>&1 || { echo "$lib trace fail"; exit 1; }
  python3 -c "
import csv; rows=[r for r in csv.DictReader(open('$OUT/trace_$n/run_kernel_stats.csv')) if 'k_conduction<' in r['Name']]
for r in rows: print('$n', r['Name'][:40], 'calls', r['Calls'], 'avg_us %.1f' % (float(r['AverageNs'])/1e3))" | tee -a $OUT/kernel_stats.txt
done
