#!/bin/bash
# after the interleaved cursors: wave end times at N = 8, and the refill / shadow-grid knobs
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; mkdir -p $OUT
export PYTHONUNBUFFERED=1
RANKS=8 timeout -k 10 200 python tools/wave_tail.py > $OUT/wt_n8.txt 2>&1 || { tail $OUT/wt_n8.txt; exit 3; }
grep -E "trace|shadow" $OUT/wt_n8.txt | cut -c1-160
RANKS=8 ROUNDS=4 VARIANTS="9=0,9=40,9=56,6=40,6=60,6=75" timeout -k 10 300 python tools/tune_ab.py > $OUT/n8.log 2>&1 || { tail $OUT/n8.log; exit 3; }
sed "s/^/N=8 /" $OUT/n8.log | grep setting
RANKS=1 ROUNDS=3 VARIANTS="9=0,9=24,9=40,6=60,6=85" timeout -k 10 300 python tools/tune_ab.py > $OUT/n1.log 2>&1 || { tail $OUT/n1.log; exit 3; }
sed "s/^/N=1 /" $OUT/n1.log | grep setting
