#!/bin/bash
# A/B of builds of the library on one GPU box, alternating processes (box-to-box variance
# cancels).  usage: tools/build_ab.sh RANKS ROUNDS lib1.so lib2.so ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
ranks=$1; rounds=$2; shift 2
for i in $(seq 1 $rounds); do
  for lib in "$@"; do
    MOBILERT_LIB=$lib RANKS=$ranks ROUNDS=3 VARIANTS="" timeout -k 10 200 python tools/tune_ab.py 2>&1 | grep setting | sed "s|^|$(basename $lib) |"
  done
done
