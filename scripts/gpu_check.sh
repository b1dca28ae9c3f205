set -o pipefail
cd $GRAFT_REPO_ROOT
echo "== rocm-smi"; timeout -k 10 60 rocm-smi --showproductname 2>&1 | head -8
echo "== gpu tests"
timeout -k 10 900 python -m pytest tests -q -x -m gpu > gpurun_out/gpu_tests.log 2>&1; echo "pytest rc=$?"
tail -30 gpurun_out/gpu_tests.log
echo "== bench 4096"
timeout -k 10 300 python bench.py --ny 4096 --nx 4096 --steps 96 --warmup 24 --no-cpu-baseline > gpurun_out/bench4096.log 2>&1; echo "rc=$?"; tail -5 gpurun_out/bench4096.log
