#!/bin/bash
# PMC passes for the rank-0 shard of an N-rank frame (tools/level_profile.py with RANKS=N).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${1:-pmc_shard}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "GRBM_GUI_ACTIVE TA_TA_BUSY TD_TD_BUSY" "TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ" "SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-include-regex "k_trace<false" --output-format csv -d $OUT/p$i -o run -- python $R/tools/level_profile.py > $OUT/p$i.log 2>&1 || { rc=$?; echo "pmc pass $i failed rc=$rc"; tail -3 $OUT/p$i.log; exit $rc; }
done
