# Round 4, ninth session: the GPU suite and the deep-launch parity cases with the
# whole-sample floors and every depletion step held to the depth's tolerance.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-r4i}
stop() { rc=$1; case $rc in 124|134|137|139) echo "GPU step ended with $rc: stopping"; exit $rc;; esac; }
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${tag}_gpu_tests.log; stop $rc; [ $rc -eq 0 ] || exit $rc
run() { name=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/${tag}_$name.json 2> gpurun_out/${tag}_$name.err
  rc=$?; echo "$name rc=$rc"; stop $rc; [ $rc -eq 0 ] || { tail -5 gpurun_out/${tag}_$name.err; return $rc; }
  python3 -c "
import json; d = json.loads([l for l in open('gpurun_out/${tag}_$name.json') if l.startswith('{')][-1]); sp = d['sample_parity']
print('$name', '%.2f G' % (d['value'] / 1e9), 'K', d['config']['fuse_steps'], 'ok', sp['ok'], 'cells', sp['cells'], 'err %.3e' % sp['max_floored_rel'], sp['max_floored_rel_at']['output'], 'flips', sp['melt_out_flips'], '/', sp['flips_fp64_baseline'], 'genuine', sp['genuine_mismatches'], 'onsets', sp.get('melt_onsets_explained'), 'depletion', sp.get('depletion_steps'), flush=True)"; }
run shard_n8 --ny 1024 --nx 8192 --steps 2304 --no-cpu-baseline --no-dropin &&
run cfg2_auto --ny 1024 --nx 1024 --steps 2304 --no-cpu-baseline --no-dropin &&
run bench_driver --gpus 1 --steps 20 --warmup 5
