# Round 5: the final-code record after the fp64 quotient folds (gpu_r5_final_c.sh: GPU suite with
# TFG_REPORT_DIR, fp64 PMC profile, bench line, issue counters of both engines, smoke).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5s} bash scripts/gpu_r5_final_c.sh
