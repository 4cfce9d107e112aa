#!/bin/bash
# A/B of prebuilt libraries at the N = 8, 4, 2 shards and N = 1, alternating processes.
# usage: tools/_ab_libs4.sh OUTNAME "lib1 lib2 ..." [ROUNDS]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; mkdir -p $OUT
export PYTHONUNBUFFERED=1
for ranks in 8 4 2 1; do for rep in 1 2; do for lib in $2; do
  MOBILERT_LIB=ab/$lib.so RANKS=$ranks ROUNDS=${3:-3} VARIANTS="" timeout -k 10 200 python tools/tune_ab.py > $OUT/$lib.$ranks.$rep.log 2>&1 || { tail $OUT/$lib.$ranks.$rep.log; exit 3; }
  grep setting $OUT/$lib.$ranks.$rep.log | sed "s|^|N=$ranks $lib |"
done; done; done
