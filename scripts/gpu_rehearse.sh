# The N > 1 bench path rehearsed on a one-GPU box (every rank on cuda:0, gloo):
# `bench.py --gpus 4` starting its own four ranks (strong scaling, 2048 x 8192 per rank, --fuse 96 so that
# four ranks' history fits one card), then N = 2 launched the way the driver launches it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TFG_BENCH_BACKEND=gloo TFG_BENCH_ONE_DEVICE=1 HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/${TAG:-reh}
mkdir -p $OUT
timeout -k 10 600 python bench.py --gpus 4 --steps 20 --warmup 5 --fuse 96 --no-cpu-baseline > $OUT/n4_self.log 2>&1 || exit $?
grep '^{' $OUT/n4_self.log | cut -c1-300
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29523 \
  bench.py --gpus 2 --steps 20 --warmup 5 --fuse 96 --no-cpu-baseline > $OUT/n2_driver.log 2>&1 || exit $?
grep '^{' $OUT/n2_driver.log | cut -c1-300
