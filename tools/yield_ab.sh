#!/bin/bash
# Cooperative shadow yield (tuning key 32): invariance tests, A/B at N = 1 and the N = 8 shard on both
# stand-ins (one process per case, interleaved renderers), and the N = 1 kernel timeline with it on.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${1:-yield}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
python -c "from mobileraytracer_amd import _native as n; assert n.build_is_current(), 'stale libmobilert_amd.so'" || exit 2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread -k "yield or overlap" > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 3; }
grep -E "passed|failed" $OUT/pytest.log | tail -2
for scene in conference flat; do for ranks in 1 8; do
  SCENE=$scene RANKS=$ranks ROUNDS=${ROUNDS:-6} VARIANTS="32=0,32=1" timeout -k 10 300 python tools/tune_ab.py > $OUT/ab_${scene}_$ranks.log 2>&1 || { tail $OUT/ab_${scene}_$ranks.log; exit 4; }
  sed "s/^/$scene N=$ranks /" $OUT/ab_${scene}_$ranks.log
done; done
cd /tmp && export TMPDIR=/tmp
MRT_BENCH_TUNING=32=1 timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $OUT/tl -o run -- python $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline > $OUT/tl.log 2>&1 || { tail $OUT/tl.log; exit 5; }
f=$(find $OUT/tl -name "*kernel_trace.csv" | head -1); python $R/tools/trace_frame.py $f > $OUT/n1_yield.timeline; cat $OUT/n1_yield.timeline
echo yield-done
