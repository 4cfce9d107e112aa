#!/bin/bash
# refill threshold sweep at HEAD (tuning key 9; 0 = auto: 32, 48 below 4 paths per lane)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; mkdir -p $OUT
export PYTHONUNBUFFERED=1
RANKS=1 ROUNDS=4 VARIANTS="9=0,9=24,9=28,9=40" timeout -k 10 300 python tools/tune_ab.py > $OUT/n1.log 2>&1 || { tail $OUT/n1.log; exit 3; }
sed "s/^/N=1 /" $OUT/n1.log | grep setting
RANKS=8 ROUNDS=4 VARIANTS="9=0,9=32,9=40,9=56,9=64" timeout -k 10 300 python tools/tune_ab.py > $OUT/n8.log 2>&1 || { tail $OUT/n8.log; exit 3; }
sed "s/^/N=8 /" $OUT/n8.log | grep setting
