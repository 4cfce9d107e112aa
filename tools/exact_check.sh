#!/bin/bash
# Exact cull mode: adversarial + full-frame parity tests, then C4 timing / counts per cull mode.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-exact}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_cull_exactness.py tests/test_full_frame.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -25 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
VARIANTS=${VARIANTS:-2=3,2=0,2=1} bash tools/cull_measure.sh ${1:-exact}
