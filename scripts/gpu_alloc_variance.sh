# Rate across fresh allocations in one process (tests/diagnostics/alloc_variance.py),
# for plane strides n_pad + skew (TFG_PLANE_SKEW, cells; "default" = the library's own),
# per shape "ny nx K reps" (SHAPES separated by ';'), and per TFG_ARENA value (ARENAS,
# default "0": 1 = forcing, window and output planes in one allocation).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/alloc_var; mkdir -p $OUT
IFS=';' read -ra SH <<< "${SHAPES:-4096 4096 192 8}"
for shape in "${SH[@]}"; do
  set -- $shape
  for ar in ${ARENAS:-0}; do
  export TFG_ARENA=$ar
  for sk in ${SKEWS:-0 1024 16384 262144}; do
    if [ "$sk" = default ]; then unset TFG_PLANE_SKEW; else export TFG_PLANE_SKEW=$sk; fi
    timeout -k 10 300 python tests/diagnostics/alloc_variance.py $1 $2 $3 $4 > $OUT/${1}x${2}_a${ar}_skew$sk.jsonl 2>$OUT/${1}x${2}_a${ar}_skew$sk.err || { tail -3 $OUT/${1}x${2}_a${ar}_skew$sk.err; exit 1; }
    python3 -c "
import json; v=[json.loads(l)['G_cell_updates_s_steady'] for l in open('$OUT/${1}x${2}_a${ar}_skew$sk.jsonl')]
print('$1x$2 K=$3 arena $ar skew $sk', ' '.join('%.1f'%x for x in v), 'mean %.1f min %.1f'%(sum(v)/len(v), min(v)))"
  done
  done
done
