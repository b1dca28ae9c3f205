# Round 4: PMC traffic profiles of both engines' timed kernels with the
# calibration passes working (tools/hbm_mix cal: 4, 8 and 16 B lanes), installed
# under profiles/ on the box so that the bench lines that follow quote them.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-r4pmc}
PMC_TAG=${tag}_f32 PMC_PROFILE=gpurun_out/${tag}_pmc_8192x8192_fuse128.json bash scripts/gpu_pmc.sh || exit $?
cp gpurun_out/${tag}_pmc_8192x8192_fuse128.json profiles/pmc_8192x8192_fuse128.json
PMC_TAG=${tag}_f64 PMC_ENGINE=float64 PMC_SHAPE="4096 4096 192" \
  PMC_ARGS="--ny 4096 --nx 4096 --engine float64 --fuse 192 --steps 1152 --warmup 192 --no-cpu-baseline --no-dropin --no-parity" \
  PMC_PROFILE=gpurun_out/${tag}_pmc_4096x4096_fuse192_f64.json bash scripts/gpu_pmc.sh || exit $?
cp gpurun_out/${tag}_pmc_4096x4096_fuse192_f64.json profiles/pmc_4096x4096_fuse192_f64.json
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${tag}_bench_driver.json 2> gpurun_out/${tag}_bench_driver.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --ny 4096 --nx 4096 --engine float64 --no-cpu-baseline --no-dropin > gpurun_out/${tag}_bench_f64.json 2> gpurun_out/${tag}_bench_f64.err
rc=$?; echo "bench f64 rc=$rc"; [ $rc -eq 0 ] || exit $rc
for f in bench_driver bench_f64; do
  python3 -c "
import json; d = json.loads([l for l in open('gpurun_out/${tag}_$f.json') if l.startswith('{')][-1]); r = d['roofline']
print('$f', '%.2f G' % (d['value'] / 1e9), 'frac %.4f' % r['frac'], 'traffic', r['traffic'], r['traffic_source'].get('match'), 'parity', d['sample_parity']['ok'])"
done
