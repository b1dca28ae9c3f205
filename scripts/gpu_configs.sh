# BASELINE configs 2/3 and the fp64 engine, one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { timeout -k 10 600 python bench.py "$@" --no-pcie > gpurun_out/cfg.log 2>&1 || { tail -3 gpurun_out/cfg.log; return 1; }
        python -c "import json; r=json.loads(open('gpurun_out/cfg.log').read().strip().splitlines()[-1]); c=r.get('cpu_baseline') or {}; print('$*', '| %.4e cell-updates/s'%r['value'], '| %.0f GB/s'%r['roofline']['achieved'], '| cpu %.3e'%c.get('value', 0), '| parity', r.get('sample_parity'))"; }
run --ny 1024 --nx 1024 --steps 960 &&
run --ny 4096 --nx 4096 --steps 480 &&
run --ny 4096 --nx 4096 --steps 96 --engine float64 --fuse 24 &&
run --ny 8192 --nx 8192 --steps 96 --engine float64 --fuse 24 --no-cpu-baseline
