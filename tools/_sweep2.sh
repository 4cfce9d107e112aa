#!/bin/bash
# level 1 at N = 8: fused packet walk + shading (default) vs the packet walk with k_shade (17=0) vs
# the per-lane walk (16=0); and the refill threshold (key 9)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; mkdir -p $OUT
export PYTHONUNBUFFERED=1
RANKS=8 ROUNDS=4 VARIANTS="16=1,17=0,16=0,9=32,9=64" timeout -k 10 300 python tools/tune_ab.py > $OUT/n8.log 2>&1 || { tail $OUT/n8.log; exit 3; }
sed "s/^/N=8 /" $OUT/n8.log | grep setting
RANKS=4 ROUNDS=4 VARIANTS="16=1,17=0,16=0" timeout -k 10 300 python tools/tune_ab.py > $OUT/n4.log 2>&1 || { tail $OUT/n4.log; exit 3; }
sed "s/^/N=4 /" $OUT/n4.log | grep setting
RANKS=1 ROUNDS=3 VARIANTS="9=0,9=24,9=40,16=0" timeout -k 10 300 python tools/tune_ab.py > $OUT/n1.log 2>&1 || { tail $OUT/n1.log; exit 3; }
sed "s/^/N=1 /" $OUT/n1.log | grep setting
