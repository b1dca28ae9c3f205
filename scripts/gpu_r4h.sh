# Round 4, eighth session: the deep-launch parity cases with the melt-onset and
# depletion rules of the GPU suite (config 2 at K = 384, the N = 8 and N = 4
# shards, config 5's slab), then the driver's bench command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-r4h}
stop() { rc=$1; case $rc in 124|134|137|139) echo "GPU step ended with $rc: stopping"; exit $rc;; esac; }
run() { name=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/${tag}_$name.json 2> gpurun_out/${tag}_$name.err
  rc=$?; echo "$name rc=$rc"; stop $rc; [ $rc -eq 0 ] || { tail -5 gpurun_out/${tag}_$name.err; return $rc; }
  python3 -c "
import json; d = json.loads([l for l in open('gpurun_out/${tag}_$name.json') if l.startswith('{')][-1]); sp = d['sample_parity']
print('$name', '%.2f G' % (d['value'] / 1e9), 'K', d['config']['fuse_steps'], 'ok', sp['ok'], 'cells', sp['cells'], 'err %.2e' % sp['max_floored_rel'], 'flips', sp['melt_out_flips'], '/', sp['flips_fp64_baseline'], 'genuine', sp['genuine_mismatches'], 'onsets', sp.get('melt_onsets_explained'), 'depletion', sp.get('depletion_steps'), 'first launches', d['launches']['ms_each'][:3], flush=True)"; }
run cfg2_auto --ny 1024 --nx 1024 --steps 2304 --no-cpu-baseline --no-dropin &&
run shard_n8 --ny 1024 --nx 8192 --steps 2304 --no-cpu-baseline --no-dropin &&
run shard_n4 --ny 2048 --nx 8192 --steps 2304 --no-cpu-baseline --no-dropin &&
run cfg5_slab --ny 2048 --nx 16384 --dt 0.25 --catchments 43 --steps 2304 --no-cpu-baseline --no-dropin &&
run bench_driver --gpus 1 --steps 20 --warmup 5
