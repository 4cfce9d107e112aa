#!/bin/bash
# packet-walk A/B: parity subset on the in-tree build, level profile, then ab/<base>.so vs ab/<new>.so
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-pk}; base=${2:-pk}; new=${3:-pk2}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_full_frame.py tests/test_cull_exactness.py tests/test_gpu_parity.py -k "packet or full or exact or walks_are" > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 3; }
tail -2 $OUT/t.log
timeout -k 10 200 python -u tools/level_profile.py > $OUT/levels.log 2>&1 || exit 4
head -4 $OUT/levels.log
AB_NAME=$1 bash tools/ab3.sh $base $new
