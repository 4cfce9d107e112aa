#!/bin/bash
# level 1 fused (17=1, default) or separate launches (17=0) by shard size
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; mkdir -p $OUT
export PYTHONUNBUFFERED=1
for n in 8 4 2; do
RANKS=$n ROUNDS=6 VARIANTS="17=1,17=0" timeout -k 10 300 python tools/tune_ab.py > $OUT/n$n.log 2>&1 || { tail $OUT/n$n.log; exit 3; }
sed "s/^/N=$n /" $OUT/n$n.log | grep setting
done
