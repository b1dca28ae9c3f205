# Same-box A/B: k_fused stepping only the cells (default) against stepping the
# whole plane stride with its skew (diag_libs/_tfg_stepskew.so, -DTFG_STEP_SKEW=1:
# the round-3 kernel, code hash f328b2f9), alternating, at each shape in SHAPES.
# One bench.py line per run (no parity / CPU / drop-in legs), summarised per run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-skew}
i=0
for shape in ${SHAPES:-"8192,8192,0" "1024,1024,120" "4096,4096,0"}; do
  IFS=, read ny nx k <<< "$shape"
  for v in base step base step base step; do
    i=$((i+1))
    lib=topoflow-glacier_amd/topoflow_glacier/_tfg.so
    [ "$v" = base ] || lib=diag_libs/_tfg_stepskew.so
    steps=2304; [ "$k" = 0 ] || steps=$((k * 24))
    TFG_LIB=$lib timeout -k 10 300 python -u bench.py --ny $ny --nx $nx --fuse $k --steps $steps --warmup 0 \
        --no-cpu-baseline --no-dropin --no-parity > gpurun_out/${tag}_${i}_${ny}_${v}.json 2> gpurun_out/${tag}_${i}_${ny}_${v}.err
    rc=$?
    case $rc in 0) ;; 124|134|137|139) echo "GPU step ended with $rc: stopping"; exit $rc;; *) tail -3 gpurun_out/${tag}_${i}_${ny}_${v}.err; exit $rc;; esac
    python3 -c "
import json; d = json.loads([l for l in open('gpurun_out/${tag}_${i}_${ny}_${v}.json') if l.startswith('{')][-1])
print('${ny}x${nx}', '$v', 'K', d['config']['fuse_steps'], '%.2f G' % (d['value'] / 1e9), 'frac %.4f' % d['roofline']['frac'], 'ms/launch %.3f' % d['roofline']['kernel_ms_per_launch'], flush=True)"
  done
done
