#!/bin/bash
# Memory-pipeline PMC passes (TA / TD / TCP) on the closest-hit trace kernel, one group per run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${1:-pmc_deep}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
CMD="python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline"
i=0
for grp in "GRBM_GUI_ACTIVE TA_TA_BUSY TD_TD_BUSY" "TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES" \
           "TCP_TCP_LATENCY TCP_TCC_READ_REQ_LATENCY" "TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES TA_FLAT_READ_WAVEFRONTS" \
           "TCP_READ_TAGCONFLICT_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES TD_TC_STALL" "TA_BUSY_avr TA_BUSY_max GRBM_TA_BUSY"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-include-regex "k_trace<false" --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1 || { rc=$?; echo "pmc pass $i ($grp) failed rc=$rc"; tail -3 $OUT/p$i.log; exit $rc; }
done
