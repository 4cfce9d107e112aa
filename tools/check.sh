#!/bin/bash
# The GPU test suite (optionally a -k selection), then the bench line.
# usage: tools/check.sh NAME [pytest -k expression]
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd)
OUT=$R/gpurun_out/${1:-check}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
python -c "from mobileraytracer_amd import _native as n; assert n.build_is_current(), 'stale libmobilert_amd.so'" || exit 2
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread ${2:+-k "$2"} > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/pytest_gpu.log | tail -15
  [ $rc -ne 0 ] && exit $rc
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  timeout -k 10 300 python bench.py ${BENCH_ARGS:---no-cpu-baseline} > $OUT/bench.log 2>&1 || { echo bench failed; tail $OUT/bench.log; exit 4; }
  tail -1 $OUT/bench.log > $OUT/bench.json; cut -c1-400 $OUT/bench.json
fi
if [ -n "${THEN:-}" ]; then bash -c "$THEN" || exit 5; fi
echo check-done
