# Round 4: the work-queue launch (TFG_WQ=1): its bit-exactness test, the GPU
# parity tests that fuse several launches run in work-queue mode, then the A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-r4w}
stop() { rc=$1; case $rc in 124|134|137|139) echo "GPU step ended with $rc: stopping"; exit $rc;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v -m gpu -x --timeout 120 --timeout-method thread \
    -k "work_queue" > gpurun_out/${tag}_wq_test.log 2>&1
rc=$?; echo "wq test rc=$rc"; tail -4 gpurun_out/${tag}_wq_test.log; stop $rc; [ $rc -eq 0 ] || exit $rc
TFG_WQ=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -v -m gpu -x --timeout 120 --timeout-method thread \
    -k "synthetic_vs_oracle or fusion_is_invisible or launches_longer or row_shards or plane_stride or checkpoint" \
    > gpurun_out/${tag}_parity_wq.log 2>&1
rc=$?; echo "parity in wq mode rc=$rc"; tail -3 gpurun_out/${tag}_parity_wq.log; stop $rc; [ $rc -eq 0 ] || exit $rc
TAG=${tag}_ab bash scripts/gpu_ab_wq.sh
