#!/bin/bash
# Round 4: parity tests, the bench line, and the shadow stream's hardware-queue probe (render stream
# and shadow stream with or without an RCCL process group created first, per shadow priority).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd)
OUT=$R/gpurun_out/${1:-r4}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
python -c "from mobileraytracer_amd import _native as n; assert n.build_is_current(), 'stale libmobilert_amd.so'" || exit 2
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread ${2:+-k "$2"} > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/pytest_gpu.log | tail -15
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo bench failed; tail $OUT/bench.log; exit 4; }
tail -1 $OUT/bench.log > $OUT/bench.json; cut -c1-400 $OUT/bench.json
if [ "${PROBE:-1}" = "1" ]; then
  unset GPU_MAX_HW_QUEUES
  for f in "" "--pg-first" "--extra-streams 1" "--extra-streams 2" "--extra-streams 3" "--pg-first --extra-streams 3"; do
    timeout -k 10 120 python tools/stream_probe.py $f >> $OUT/probe.log 2>&1 || { echo probe failed; tail $OUT/probe.log; exit 5; }
    echo "$f $(tail -1 $OUT/probe.log)"
  done
fi
