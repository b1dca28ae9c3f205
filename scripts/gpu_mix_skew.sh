# The bare streaming ceiling of k_fused's access mix (tools/hbm_mix: 6 read and
# 7 write planes, 4 B lanes) at plane skews 0 and 512 cells, 2^26 cells, 3 runs each.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/mix_skew; mkdir -p $OUT
for rep in 1 2 3; do
  for sk in 0 512; do
    timeout -k 10 120 tools/hbm_mix 67108864 24 32768 $sk > $OUT/mix_${sk}_$rep.json 2>&1 || { tail -3 $OUT/mix_${sk}_$rep.json; exit 1; }
    echo "skew=$sk rep=$rep $(head -c 400 $OUT/mix_${sk}_$rep.json | tr '\n' ' ')"
  done
done
