# Round 4, final profile set on the final code: rocprofv3 kernel trace + stats of
# the driver's bench command and its summary, smoke, the bench line with no
# flags, a world-size-1 RCCL bench line (TFG_BENCH_PG=1: the N > 1 barrier,
# max-over-ranks and diagnostics all-reduce over RCCL), and the 4-rank gloo
# rehearsal of the N > 1 path on one GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-r4k}
stop() { rc=$1; case $rc in 124|134|137|139) echo "GPU step ended with $rc: stopping"; exit $rc;; esac; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_trace -o run --output-format csv -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${tag}_bench_traced.log 2> gpurun_out/${tag}_bench_traced.err
rc=$?; echo "traced bench rc=$rc"; stop $rc; [ $rc -eq 0 ] || { tail -5 gpurun_out/${tag}_bench_traced.err; exit $rc; }
python3 scripts/trace_summary.py gpurun_out/${tag}_trace gpurun_out/${tag}_bench_traced.log gpurun_out/${tag}_trace_summary.json | tail -3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${tag}_smoke.log; stop $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/${tag}_bench_default.json 2> gpurun_out/${tag}_bench_default.err
rc=$?; echo "bench default rc=$rc"; stop $rc; [ $rc -eq 0 ] || exit $rc
TFG_BENCH_PG=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-dropin \
    > gpurun_out/${tag}_bench_rccl_world1.json 2> gpurun_out/${tag}_bench_rccl_world1.err
rc=$?; echo "bench rccl world1 rc=$rc"; stop $rc; [ $rc -eq 0 ] || { tail -5 gpurun_out/${tag}_bench_rccl_world1.err; exit $rc; }
export TFG_BENCH_BACKEND=gloo TFG_BENCH_ONE_DEVICE=1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29521 \
  bench.py --gpus 4 --steps 20 --warmup 5 --fuse 96 --no-cpu-baseline > gpurun_out/${tag}_rehearse4_strong.json 2> gpurun_out/${tag}_rehearse4_strong.err
rc=$?; echo "rehearse4 rc=$rc"; stop $rc
for f in bench_default bench_rccl_world1 rehearse4_strong; do
  python3 -c "
import json; d = json.loads([l for l in open('gpurun_out/${tag}_$f.json') if l.startswith('{')][-1]); sp = d['sample_parity']
print('$f', '%.2f G' % (d['value'] / 1e9), 'pg', d['process_group'], 'parity ok', sp['ok'], 'err %.3e' % sp['max_floored_rel'])" || true
done
