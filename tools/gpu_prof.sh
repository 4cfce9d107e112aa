#!/bin/bash
# Bench + rocprofv3 kernel stats of the serialised bench (the roofline's durations) + PMC passes.
# usage: tools/gpu_prof.sh NAME
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${1:-prof}; mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { echo bench failed; tail $OUT/bench.log; exit 4; }
tail -1 $OUT/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_serial -o run --output-format csv -- python $R/bench.py --steps 5 --warmup 1 --overlap 0 --no-cpu-baseline > $OUT/prof_serial.log 2>&1 || { echo rocprof failed; tail $OUT/prof_serial.log; exit 5; }
tail -1 $OUT/prof_serial.log
cd $R && bash tools/pmc_run.sh ${1:-prof}/pmc
