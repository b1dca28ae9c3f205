# Round 5: the parity samples of every rank of the strong-scaling lines (8192^2 split over N ranks),
# each run on this one GPU as its own process (tests/diagnostics/parity_tail.py --rank R --world N).
# RANKS: "N:R ..." pairs.  TAG names the outputs.  LIB=<path> runs a variant library (TFG_LIB).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-r5rank}
[ -n "$LIB" ] && export TFG_LIB=$PWD/$LIB
for pr in ${RANKS:-2:1 4:1 4:2 4:3 8:1 8:2 8:3 8:4 8:5 8:6 8:7}; do
  n=${pr%%:*}; r=${pr##*:}
  timeout -k 10 300 python -u tests/diagnostics/parity_tail.py gpurun_out/${tag}_n${n}r${r}.npz 64 --rank $r --world $n \
    -- --ny 8192 --nx 8192 > gpurun_out/${tag}_n${n}r${r}.log 2>&1
  rc=$?; echo "N=$n rank $r rc=$rc $(tail -1 gpurun_out/${tag}_n${n}r${r}.log)"
  case $rc in 0) ;; *) exit $rc;; esac
done
