# Round 4: the BMI scalar fast paths: the GPU suite (every BMI, caller and
# defer_update test), then the bench with its drop-in legs (defer_update
# instances fed numpy scalars, as the reference's driver).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-r4bmi}
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${tag}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${tag}_bench_driver.json 2> gpurun_out/${tag}_bench_driver.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "
import json; d = json.loads([l for l in open('gpurun_out/${tag}_bench_driver.json') if l.startswith('{')][-1])
print('%.2f G' % (d['value'] / 1e9), 'parity', d['sample_parity']['ok'], json.dumps(d['dropin_defer_update_instances']), json.dumps(d['dropin_per_step_grid']['per_step']))"
