# Same-box A/B of the work-queue launch (TFG_WQ=1: the steps of one engine call
# as ONE launch whose resident workgroups pull (chunk, range) items from per-XCD
# queues) against one launch per range (TFG_WQ=0), the same library, alternating;
# bench.py --one-call (every timed step in one engine call) in both arms.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-wq}
i=0
for shape in ${SHAPES:-"1024,1024,120,2880" "1024,1024,0,2304" "1024,8192,384,2304" "8192,8192,0,2304"}; do
  IFS=, read ny nx k steps <<< "$shape"
  for wq in 0 1 0 1; do
    i=$((i+1))
    TFG_WQ=$wq timeout -k 10 300 python -u bench.py --ny $ny --nx $nx --fuse $k --steps $steps --warmup 0 --one-call \
        --no-cpu-baseline --no-dropin --no-parity > gpurun_out/${tag}_${i}_${ny}x${nx}_wq$wq.json 2> gpurun_out/${tag}_${i}_${ny}x${nx}_wq$wq.err
    rc=$?
    case $rc in 0) ;; 124|134|137|139) echo "GPU step ended with $rc: stopping"; exit $rc;; *) tail -3 gpurun_out/${tag}_${i}_${ny}x${nx}_wq$wq.err; exit $rc;; esac
    python3 -c "
import json; d = json.loads([l for l in open('gpurun_out/${tag}_${i}_${ny}x${nx}_wq$wq.json') if l.startswith('{')][-1])
print('${ny}x${nx}', 'wq$wq', 'K', d['config']['fuse_steps'], '%.2f G' % (d['value'] / 1e9), 'frac %.4f' % d['roofline']['frac'], flush=True)"
  done
done
