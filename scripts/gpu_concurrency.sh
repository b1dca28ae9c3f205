# Same box: one process vs two processes sharing the GPU (equal total cells).
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
one() { timeout -k 10 300 python bench.py --ny $1 --nx 8192 --steps 192 --no-cpu-baseline --no-pcie > gpurun_out/c1.log 2>&1 || return 1
        python -c "import json; r=json.loads(open('gpurun_out/c1.log').read().strip().splitlines()[-1]); print('1 proc ny=$1', '%.3e'%r['value'], 'ms/launch %.2f'%r['roofline']['kernel_ms_per_launch'])"; }
two() { TFG_BENCH_BACKEND=gloo TFG_BENCH_ONE_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
          --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --ny $1 --nx 8192 --steps 192 --no-cpu-baseline --no-pcie > gpurun_out/c2.log 2>&1 || return 1
        python -c "import json; r=[l for l in open('gpurun_out/c2.log').read().splitlines() if l.startswith('{')][-1]; r=json.loads(r); print('2 proc ny=$1 each', '%.3e'%r['value'], 'ms/launch %.2f'%r['roofline']['kernel_ms_per_launch'])"; }
one 4096 && two 2048 && one 2048 && one 4096 && two 2048
