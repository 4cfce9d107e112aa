#!/bin/bash
# Cull modes 0/1/2 on the current walk: C4 frame time (N=1 and the N=8 shard) and counting stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-cull}
mkdir -p $OUT
V=${VARIANTS:-2=1,2=0,2=2}
VARIANTS=$V ROUNDS=3 timeout -k 10 300 python -u tools/tune_ab.py > $OUT/n1.log 2>&1 || { cat $OUT/n1.log; exit 3; }
cat $OUT/n1.log
RANKS=8 VARIANTS=$V ROUNDS=3 timeout -k 10 300 python -u tools/tune_ab.py > $OUT/n8.log 2>&1 || { cat $OUT/n8.log; exit 4; }
cat $OUT/n8.log
VARIANTS=$V timeout -k 10 300 python -u tools/count_ab.py > $OUT/count.log 2>&1 || { cat $OUT/count.log; exit 5; }
cat $OUT/count.log
