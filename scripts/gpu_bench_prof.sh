set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -3 gpurun_out/smoke.log
echo "== bench default"
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1; echo "bench rc=$?"; tail -2 gpurun_out/bench_default.log
echo "== rocprof kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1 -o run --output-format csv -- python bench.py --steps 96 --no-cpu-baseline > gpurun_out/prof_r1.log 2>&1; echo "prof rc=$?"
find gpurun_out/prof_r1 -name "*stats*" | head
