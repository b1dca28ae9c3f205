# Round 4, fifth session: per-workgroup timelines of config 2 at launch depths
# 120-3840 and of the headline shape; config 2 at its automatic depth (bounded
# parity sample); the fp64 engine's bench line (PMC traffic quoted by hash);
# the rocprofv3 kernel trace of the driver's bench command; smoke.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-r4e}
stop() { rc=$1; case $rc in 124|134|137|139) echo "GPU step ended with $rc: stopping"; exit $rc;; esac; }
TFG_LIB=diag_libs/_tfg_wgt.so timeout -k 10 400 python -u tests/diagnostics/wg_timeline.py gpurun_out/${tag}_wg_timeline.json \
    1024,1024,120 1024,1024,480 1024,1024,1920 1024,1024,3840 8192,8192,128 > gpurun_out/${tag}_wg_timeline.log 2>&1
rc=$?; echo "timeline rc=$rc"; stop $rc; [ $rc -eq 0 ] || { tail -5 gpurun_out/${tag}_wg_timeline.log; exit $rc; }
timeout -k 10 400 python -u bench.py --ny 1024 --nx 1024 --steps 2304 --no-cpu-baseline --no-dropin \
    > gpurun_out/${tag}_cfg2_auto.json 2> gpurun_out/${tag}_cfg2_auto.err
rc=$?; echo "cfg2 auto rc=$rc"; stop $rc; [ $rc -eq 0 ] || { tail -5 gpurun_out/${tag}_cfg2_auto.err; exit $rc; }
timeout -k 10 400 python -u bench.py --ny 4096 --nx 4096 --engine float64 --no-cpu-baseline --no-dropin \
    > gpurun_out/${tag}_bench_f64.json 2> gpurun_out/${tag}_bench_f64.err
rc=$?; echo "bench f64 rc=$rc"; stop $rc; [ $rc -eq 0 ] || { tail -5 gpurun_out/${tag}_bench_f64.err; exit $rc; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_trace -o run --output-format csv -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${tag}_bench_traced.log 2> gpurun_out/${tag}_bench_traced.err
rc=$?; echo "traced bench rc=$rc"; stop $rc; [ $rc -eq 0 ] || { tail -5 gpurun_out/${tag}_bench_traced.err; exit $rc; }
python3 scripts/trace_summary.py gpurun_out/${tag}_trace gpurun_out/${tag}_bench_traced.log gpurun_out/${tag}_trace_summary.json | tail -3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${tag}_smoke.log
