cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1; echo rc=$?
grep -oE "^[ ]*(SQ_[A-Z_0-9]+|TCC_[A-Z_0-9]+|TCP_[A-Z_0-9]+|GRBM_[A-Z_0-9]+|FETCH_SIZE|WRITE_SIZE|VALUBusy|MemUnitBusy|OccupancyPercent|VALUUtilization|MemUnitStalled|Wavefronts)" gpurun_out/counters_list.txt | sort -u | tr -d ' ' | tr '\n' ' ' | head -c 6000
