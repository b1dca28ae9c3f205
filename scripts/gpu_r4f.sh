# Round 4, sixth session: parity of the deeper launches the driver's N > 1 lines
# time (each rank's shard run alone at N = 1: 4096 x 8192 at K = 256, 1024 x 8192
# at K = 384, config 5's 2048 x 16384 slab at K = 256), config 2 at K = 384, with
# the first genuine mismatches kept in the line; raw per-workgroup timelines of
# config 2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-r4f}
stop() { rc=$1; case $rc in 124|134|137|139) echo "GPU step ended with $rc: stopping"; exit $rc;; esac; }
run() { name=$1; shift
  timeout -k 10 400 python -u bench.py "$@" --no-cpu-baseline --no-dropin > gpurun_out/${tag}_$name.json 2> gpurun_out/${tag}_$name.err
  rc=$?; echo "$name rc=$rc"; stop $rc; [ $rc -eq 0 ] || { tail -5 gpurun_out/${tag}_$name.err; return $rc; }
  python3 -c "
import json; d = json.loads([l for l in open('gpurun_out/${tag}_$name.json') if l.startswith('{')][-1]); sp = d['sample_parity']
print('$name', '%.2f G' % (d['value'] / 1e9), 'K', d['config']['fuse_steps'], 'ok', sp['ok'], 'cells', sp['cells'], 'err %.2e' % sp['max_floored_rel'], 'flips', sp['melt_out_flips'], '/', sp['flips_fp64_baseline'], 'genuine', sp['genuine_mismatches'], flush=True)"; }
run cfg2_auto --ny 1024 --nx 1024 --steps 2304 &&
run shard_n2 --ny 4096 --nx 8192 --steps 2304 &&
run shard_n8 --ny 1024 --nx 8192 --steps 2304 &&
run cfg5_slab --ny 2048 --nx 16384 --dt 0.25 --catchments 43 --steps 2304 || exit 1
TFG_WG_RAW=1 TFG_LIB=diag_libs/_tfg_wgt.so timeout -k 10 300 python -u tests/diagnostics/wg_timeline.py gpurun_out/${tag}_wg_timeline_raw.json \
    1024,1024,120 1024,1024,1920 > gpurun_out/${tag}_wg_timeline.log 2>&1
echo "timeline rc=$?"
