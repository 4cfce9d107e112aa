#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-packet}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_cull_exactness.py tests/test_full_frame.py tests/test_device_kat.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
V1="16=1,16=0" bash tools/knob_sweep.sh ${1:-packet}
