# Rehearse the N>1 bench path with 4 ranks on a one-GPU box (all on cuda:0, gloo):
# the default (strong scaling: ONE 8192 x 8192 grid split 4 ways, 2048 x 8192 per
# rank) and weak scaling behind its flag (8192 rows per rank is too much memory
# for 4 ranks on one card, so 2048 rows each).  --fuse 96: four ranks' 192-step
# history (4 x 77 GB) would not fit one card's 288 GB; on the driver's node each
# rank has its own GPU and the automatic depth.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TFG_BENCH_BACKEND=gloo TFG_BENCH_ONE_DEVICE=1 HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/${TAG:-rehearse4}
mkdir -p $OUT
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29521 \
  bench.py --gpus 4 --steps 20 --warmup 5 --fuse 96 --no-cpu-baseline > $OUT/strong.log 2>&1 || exit $?
grep '^{' $OUT/strong.log | cut -c1-600
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29519 \
  bench.py --gpus 4 --scaling weak --ny 2048 --nx 8192 --steps 20 --warmup 5 --fuse 96 --no-cpu-baseline > $OUT/weak.log 2>&1 || exit $?
grep '^{' $OUT/weak.log | cut -c1-600
