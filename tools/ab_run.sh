#!/bin/bash
# In-process A/B of tuning settings (tools/tune_ab.py) at N = 1 and the N = 8 shard, with counting
# stats.  usage: tools/ab_run.sh NAME "VARIANTS" [ROUNDS]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; mkdir -p $OUT
export PYTHONUNBUFFERED=1
for ranks in 1 8; do
  RANKS=$ranks ROUNDS=${3:-5} COUNT=1 VARIANTS="$2" timeout -k 10 300 python tools/tune_ab.py > $OUT/n$ranks.log 2>&1 || { tail $OUT/n$ranks.log; exit 3; }
  sed "s/^/N=$ranks /" $OUT/n$ranks.log
done
