# Same-box A/B of library variants (abvar/*.so) on the strong-scaling shapes as
# the driver times them (--steps 20 --warmup 5): the 1024 x 8192 slab (N = 8)
# and the whole 8192^2 grid (N = 1), alternating A B A B.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/ab_slab; mkdir -p $OUT
for rep in 1 2; do
  for lib in ${AB_LIBS:-abvar/*.so}; do
    for rows in ${ROWS:-1024 8192}; do
      TFG_LIB=$PWD/$lib timeout -k 10 300 python bench.py --ny $rows --nx 8192 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/run.log 2>&1 || { echo "$lib $rows fail"; tail -3 $OUT/run.log; exit 1; }
      python3 -c "import json; r=json.loads([l for l in open('$OUT/run.log') if l.startswith('{')][-1]); L=r['launches']; print('$lib', 'rows=$rows', 'G=%.2f'%(r['value']/1e9), 'ms min/mean %.2f/%.2f'%(L['ms_min'], L['ms_mean']))"
    done
  done
done
