# Rehearse the N>1 bench path with 4 ranks on a one-GPU box (all on cuda:0, gloo):
# weak scaling (2048 rows per rank) and strong scaling (one 8192-row grid split 4 ways).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TFG_BENCH_BACKEND=gloo TFG_BENCH_ONE_DEVICE=1 HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/rehearse4
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29519 \
  bench.py --gpus 4 --ny 2048 --nx 8192 --steps 192 --no-cpu-baseline --no-pcie > gpurun_out/rehearse4/weak.log 2>&1 || exit $?
grep '^{' gpurun_out/rehearse4/weak.log | cut -c1-420
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29521 \
  bench.py --gpus 4 --scaling strong --ny 8192 --nx 8192 --steps 192 --no-cpu-baseline --no-pcie > gpurun_out/rehearse4/strong.log 2>&1 || exit $?
grep '^{' gpurun_out/rehearse4/strong.log | cut -c1-420
