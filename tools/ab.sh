#!/bin/bash
# A/B of library builds (ab/*.so) on the conference and flat stand-ins, at N = 1 and the N = 8
# shard, alternating processes.  usage: tools/ab.sh NAME ROUNDS lib1.so lib2.so ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; mkdir -p $OUT; rounds=$2; shift 2
for scene in ${SCENES:-conference flat}; do
  for ranks in ${RANKS_LIST:-1 8}; do
    SCENE=$scene bash tools/build_ab.sh $ranks $rounds "$@" > $OUT/${scene}_n$ranks.log 2>&1
    sed "s/^/$scene N=$ranks /" $OUT/${scene}_n$ranks.log
  done
done
