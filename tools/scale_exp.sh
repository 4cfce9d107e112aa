#!/bin/bash
# Shard-scaling experiments on one GPU: rank-0 shard frame time for N = 1, 2, 4, 8 under tuning variants.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-scale}
mkdir -p $OUT
timeout -k 10 200 python tools/shard_scaling.py > $OUT/default.log 2>&1 || exit 1
cat $OUT/default.log
PIPES=2 timeout -k 10 200 python tools/shard_scaling.py > $OUT/pipes2.log 2>&1 || exit 1
cat $OUT/pipes2.log
OVERLAP=2 timeout -k 10 200 python tools/shard_scaling.py > $OUT/overlap2.log 2>&1 || exit 1
cat $OUT/overlap2.log
RANKS=8 timeout -k 10 200 python tools/level_profile.py > $OUT/level8.log 2>&1 || exit 1
cat $OUT/level8.log
timeout -k 10 200 python tools/level_profile.py > $OUT/level1.log 2>&1 || exit 1
cat $OUT/level1.log
