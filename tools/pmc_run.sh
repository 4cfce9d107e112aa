#!/bin/bash
# PMC passes on the bench command (trace, shadow and shade kernels), one counter group per run
# (rocprofv3 does not split counters over passes; MI355X_MICROARCH.md "rocprofv3 PMC slots").
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${1:-pmc}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
# extra bench arguments (a workload other than C4, e.g. "--shard-of 8") after the output name
shift
CMD="python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline $*"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE TA_TA_BUSY TD_TD_BUSY" "TCP_TCC_READ_REQ TCP_TOTAL_CACHE_ACCESSES" ; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex "k_trace|k_shadow|k_shade" --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1 || { rc=$?; echo "pmc pass $i ($grp) failed rc=$rc"; tail -5 $OUT/p$i.log; exit $rc; }
done
python $R/tools/pmc_summary.py $OUT $OUT/pmc_traffic.json $*
