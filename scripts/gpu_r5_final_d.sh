# Round 5, final code after the flat-dark shortwave skip: the fp32 profile set (PMC with calibration, kernel
# trace, driver and default bench lines, smoke: gpu_r5_round.sh), then the fp64 PMC profile, bench line and
# the issue counters of both engines (gpu_r5_final_b.sh without the rank samples).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=r5fd bash scripts/gpu_r5_round.sh || exit $?
NO_RANKS=1 TAG=r5fd64 bash scripts/gpu_r5_final_b.sh
