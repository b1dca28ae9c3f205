# Round 4, last sessions: the long-wave A/B (default kernel vs TFG_LW_SPLIT=1,
# diag_libs/_tfg_lwx.so, alternating), then the final profile set of the default
# kernel (scripts/gpu_r4k.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
VARIANTS="lwx base lwx base lwx base" TAG=${TAG:-r4final}_lw bash scripts/gpu_acc_ab.sh || exit $?
TAG=${TAG:-r4final} bash scripts/gpu_r4k.sh
