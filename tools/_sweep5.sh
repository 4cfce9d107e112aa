#!/bin/bash
# shadow walk grid (key 6) after the interleaved cursors, N = 8 and N = 4 shards, 8 rounds
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; mkdir -p $OUT
export PYTHONUNBUFFERED=1
RANKS=8 ROUNDS=8 VARIANTS="6=0,6=60,6=75,6=0" timeout -k 10 300 python tools/tune_ab.py > $OUT/n8.log 2>&1 || { tail $OUT/n8.log; exit 3; }
sed "s/^/N=8 /" $OUT/n8.log | grep setting | grep -v identical
RANKS=4 ROUNDS=6 VARIANTS="6=0,6=60,6=90,6=0" timeout -k 10 300 python tools/tune_ab.py > $OUT/n4.log 2>&1 || { tail $OUT/n4.log; exit 3; }
sed "s/^/N=4 /" $OUT/n4.log | grep setting | grep -v identical
