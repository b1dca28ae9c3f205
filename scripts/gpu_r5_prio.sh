# Round 5: the fp32 step loop issuing its loads at wave priority 3 (s_setprio around fetch), or VARIANT
# against the in-tree library, same box, alternating, at the default bench workload.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
LIBS="topoflow-glacier_amd/topoflow_glacier/_tfg.so ${VARIANT:-diag_libs/_tfg_prio.so}" TAG=${TAG:-r5prio} REPS=${REPS:-3} \
  bash scripts/gpu_r5_ab.sh
