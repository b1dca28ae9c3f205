# Instruction-issue counters (rocprofv3 --pmc, one counter set per pass) of the
# fused kernel for both engines: fp32 at 8192^2 (the bench) and fp64 at 4096^2.
# Summary: scripts/issue_summary.py.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-issue}
mkdir -p $OUT
run() {  # name, bench args
  local name=$1; shift
  local i=0
  while IFS= read -r line; do
    [ -z "$line" ] && continue
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $line --output-format csv -d $OUT/$name/p$i -o run -- python3 bench.py "$@" > $OUT/$name/p$i.log 2>&1
    rc=$?; echo "$name pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/$name/p$i.log; return $rc; fi
  done <<PASSES
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE
SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32
PASSES
}
mkdir -p $OUT/f32 $OUT/f32_flux_f64 $OUT/f64
# the bench shapes (128-step launches at 8192^2, 192 at 4096^2 for fp64), timed launches only
run f32 --ny 8192 --nx 8192 --steps 256 --warmup 128 --fuse 128 --no-cpu-baseline --no-parity --no-dropin || exit 1
run f32_flux_f64 --flux fp64 --ny 8192 --nx 8192 --steps 256 --warmup 128 --fuse 128 --no-cpu-baseline --no-parity --no-dropin || exit 1
run f64 --engine float64 --ny 4096 --nx 4096 --steps 384 --warmup 192 --fuse 192 --no-cpu-baseline --no-parity --no-dropin || exit 1
python3 scripts/issue_summary.py $OUT 128 192
