#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel stats.  Stops at the first crash.
# usage: tools/gpu_check.sh NAME [pytest -k expression]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${1:-check}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rf --timeout 240 --timeout-method thread ${2:+-k "$2"} > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/pytest_gpu.log | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 3; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { echo bench failed; tail $OUT/bench.log; exit 4; }
tail -1 $OUT/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo rocprof failed; tail $OUT/prof.log; exit 5; }
find $OUT/prof -name "*stats*" | head
