#!/bin/bash
# PMC passes on the bench command (trace kernels only), each counter group in its own run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${1:-pmc}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
CMD="python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_BRANCH" ; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-include-regex "k_trace|k_shadow|k_shade" --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1 || { rc=$?; echo "pmc pass $i ($grp) failed rc=$rc"; tail -5 $OUT/p$i.log; exit $rc; }
done
ls -R $OUT | head -40
