#!/bin/bash
# Knob sweep of the default (exact) mode at N = 1 and the N = 8 shard (tools/tune_ab.py, one process per
# RANKS setting, images compared against the first variant).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-knobs}; mkdir -p $OUT
V1=${V1:-"9=0,9=16,9=24,9=32,9=40,6=50,6=70,6=85,6=100,11=14,11=28,11=40,8=0"}
VARIANTS="$V1" ROUNDS=3 timeout -k 10 500 python -u tools/tune_ab.py > $OUT/n1.log 2>&1 || { cat $OUT/n1.log; exit 3; }
cat $OUT/n1.log
RANKS=8 VARIANTS="$V1" ROUNDS=3 timeout -k 10 400 python -u tools/tune_ab.py > $OUT/n8.log 2>&1 || { cat $OUT/n8.log; exit 4; }
cat $OUT/n8.log
