#!/bin/bash
# Round-3 session: new GPU tests, bench (new fields), C5 8-way shard rehearsal, PMC passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r3}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_0_dist_rehearsal.py tests/test_gpu_parity.py -m gpu -x -v --timeout 600 --timeout-method thread -k "${2:-rehearsal or c5 or removed or shadow_order}" > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $OUT/pytest.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { tail $OUT/bench.log; exit 4; }
tail -1 $OUT/bench.log
timeout -k 10 300 python bench.py --width 3840 --height 2160 --spp 8 --shard-of 8 --steps 10 --no-cpu-baseline > $OUT/c5_shard8.log 2>&1 || { tail $OUT/c5_shard8.log; exit 5; }
tail -1 $OUT/c5_shard8.log | cut -c1-400
bash tools/pmc_run.sh ${1:-r3}_pmc
