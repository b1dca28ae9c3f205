# Rehearse the N>1 bench path on a one-GPU box: 2 ranks, both on cuda:0, gloo.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TFG_BENCH_BACKEND=gloo TFG_BENCH_ONE_DEVICE=1 HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --ny 2048 --nx 8192 --steps 192 --no-cpu-baseline --no-pcie > gpurun_out/rehearse2.log 2>&1
rc=$?; grep '^{' gpurun_out/rehearse2.log | cut -c1-600; exit $rc
