# Same-box A/B of library variants (abvar/*.so) on small grids (BASELINE
# config 2's 1024^2 and 2048^2), K = 96, alternating; stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-ab_small}; mkdir -p $OUT
for rep in 1 2; do
  for lib in ${AB_LIBS:-abvar/*.so}; do
    for g in ${GRIDS:-1024 2048}; do
      TFG_LIB=$PWD/$lib timeout -k 10 300 python bench.py --ny $g --nx $g --fuse 96 --steps 1920 --warmup 96 --no-cpu-baseline --no-pcie > $OUT/run.log 2>&1 || { echo "$lib $g bench fail"; tail -3 $OUT/run.log; exit 1; }
      python -c "import json; r=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); l=r['launches']; print('$lib', '$g', 'value=%.2f G'%(r['value']/1e9), 'ms/launch mean %.3f min %.3f'%(r['roofline']['kernel_ms_per_launch'], l['ms_min']))"
    done
  done
done
