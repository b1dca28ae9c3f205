set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fuse128
for rep in 1 2; do
  for k in ${KS:-96 128}; do
    timeout -k 10 300 python bench.py --fuse $k --steps 1152 --warmup 5 --no-cpu-baseline > gpurun_out/fuse128/k$k.log 2>&1 || { tail -5 gpurun_out/fuse128/k$k.log; exit 1; }
    python3 -c "import json; r=json.loads([l for l in open('gpurun_out/fuse128/k$k.log') if l.startswith('{')][-1]); L=r['launches']; print('K=$k', 'G=%.2f'%(r['value']/1e9), 'launches', L['count'], 'ms min/mean %.2f/%.2f'%(L['ms_min'], L['ms_mean']), 'frac %.4f'%r['roofline']['frac'])"
  done
done
