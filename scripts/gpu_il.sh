# Layout experiment: planar planes vs block-interleaved planes for the k_fused access mix.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/il
timeout -k 10 120 tools/hbm_mix 67108864 24 32768 0 il > gpurun_out/il/mix.json 2>&1; rc=$?; cat gpurun_out/il/mix.json; exit $rc
