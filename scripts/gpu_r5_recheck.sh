# Round 5: every deep-launch sample again on the final library (rank 0 of N = 2 / 4 / 8 and configs 3 / 5,
# then ranks 1..N-1), to confirm the last kernel changes left each sample's maximum where it was.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=r5re SAMPLES="n4 n2 cfg3 cfg5" bash scripts/gpu_r5_tail.sh || exit $?
TAG=r5re_rank bash scripts/gpu_r5_ranks.sh
