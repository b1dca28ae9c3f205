# Dump flux terms for several diagnostic builds (build_variants/dbg/_tfg_<tag>_term<t>.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
for tag in ${TAGS:-n1 n2}; do
  for t in ${TERMS:-0 2 3 4 5}; do
    TFG_LIB=$PWD/build_variants/dbg/_tfg_${tag}_term$t.so timeout -k 10 120 python tests/diagnostics/gpu_term_dump.py ${tag}_$t 65536 24 || exit 1
  done
done
