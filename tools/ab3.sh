#!/bin/bash
# A/B of ab/*.so builds named on the command line at N=1 and the N=8 shard, then device KATs + cull
# exactness on the last build
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${AB_NAME:-ab}; mkdir -p $OUT
libs=""; for n in "$@"; do libs="$libs ab/$n.so"; done
timeout -k 10 500 bash tools/build_ab.sh 1 2 $libs > $OUT/n1.log 2>&1 || { cat $OUT/n1.log; exit 3; }
cat $OUT/n1.log
timeout -k 10 400 bash tools/build_ab.sh 8 2 $libs > $OUT/n8.log 2>&1 || { cat $OUT/n8.log; exit 4; }
cat $OUT/n8.log
