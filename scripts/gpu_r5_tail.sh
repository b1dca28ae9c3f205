# Round 5: the tails of the deep-launch parity samples (tests/diagnostics/parity_tail.py),
# for offline classification of the entries that set max_floored_rel.
# LIB=<path> runs a variant library (TFG_LIB).  TAG names the outputs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-r5tail}
[ -n "$LIB" ] && export TFG_LIB=$PWD/$LIB
stop() { rc=$1; case $rc in 124|134|137|139) echo "GPU step ended with $rc: stopping"; exit $rc;; esac; }
tail_of() { name=$1; shift
  timeout -k 10 300 python -u tests/diagnostics/parity_tail.py gpurun_out/${tag}_$name.npz 128 -- "$@" \
    > gpurun_out/${tag}_$name.log 2>&1
  rc=$?; echo "$name rc=$rc $(tail -1 gpurun_out/${tag}_$name.log)"; stop $rc; return $rc; }
for s in ${SAMPLES:-n4 n2 n8 cfg3 cfg4 cfg5}; do
  case $s in
    n4) tail_of n4 --ny 2048 --nx 8192 ;;
    n2) tail_of n2 --ny 4096 --nx 8192 ;;
    n8) tail_of n8 --ny 1024 --nx 8192 ;;
    cfg3) tail_of cfg3 --ny 4096 --nx 4096 ;;
    cfg4) tail_of cfg4 --ny 8192 --nx 8192 ;;
    cfg5) tail_of cfg5 --ny 2048 --nx 16384 --dt 0.25 --catchments 43 ;;
  esac || exit $?
done
