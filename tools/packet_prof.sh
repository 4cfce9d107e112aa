#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-pprof}; mkdir -p $OUT
VARIANTS="16=1,16=0" timeout -k 10 300 python -u tools/count_ab.py > $OUT/count.log 2>&1 || { cat $OUT/count.log; exit 3; }
cat $OUT/count.log
timeout -k 10 200 python -u tools/level_profile.py > $OUT/levels_packet.log 2>&1 || exit 4
head -4 $OUT/levels_packet.log
