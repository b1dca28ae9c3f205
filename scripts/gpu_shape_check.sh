# The same 2^24 cells (identical synthetic inputs: global cell indices 0..2^24-1)
# as 4096 x 4096 and as 2048 x 8192, alternating on one box, 192-step launches.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/shape
for rep in 1 2 3; do
  for shape in "4096 4096" "2048 8192"; do
    set -- $shape
    timeout -k 10 300 python bench.py --ny $1 --nx $2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/shape/run.log 2>&1 || { tail -5 gpurun_out/shape/run.log; exit 1; }
    python3 -c "import json; r=json.loads([l for l in open('gpurun_out/shape/run.log') if l.startswith('{')][-1]); L=r['launches']; print('$1x$2', 'G=%.2f'%(r['value']/1e9), 'ms each', L['ms_each'])"
  done
done
