#!/bin/bash
# Kernel timeline of the last frame at N = 1 and of rank 0's N = 8 shard (rocprofv3 kernel trace).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${1:-tl}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $OUT/n1 -o run -- python $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline > $OUT/n1.log 2>&1 || { tail $OUT/n1.log; exit 3; }
timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $OUT/n8 -o run -- python $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --shard-of 8 > $OUT/n8.log 2>&1 || { tail $OUT/n8.log; exit 4; }
for n in n1 n8; do f=$(find $OUT/$n -name "*kernel_trace.csv" | head -1); python $R/tools/trace_frame.py $f > $OUT/$n.timeline; done
echo done
