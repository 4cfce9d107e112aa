#!/bin/bash
# End-of-round measurements: PMC passes (stamped and keyed by workload), the bench line, its
# rocprofv3 kernel stats (product frames, and a run whose frames all have the shadow walks
# serialised: the durations bench's roofline events measure), the N = 8 C4 shard, the 8-way C5
# shard, the flat-geometry stand-in, the kernel timelines and the walk phase occupancy.
# usage: tools/final.sh NAME [ROUND_TAG, e.g. r06]
# Back here, copy gpurun_out/NAME_pmc/pmc_traffic.json to profiles/<tag>_pmc_traffic.json (the file
# bench.PMC_PROFILE names) and the other summaries to profiles/<tag>_* before committing.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd)
N=${1:-final}; TAG=${2:-r06}; OUT=$R/gpurun_out/$N; mkdir -p $OUT
export PYTHONUNBUFFERED=1
python -c "from mobileraytracer_amd import _native as n; assert n.build_is_current(), 'stale libmobilert_amd.so'" || exit 2
bash tools/pmc_run.sh ${N}_pmc > $OUT/pmc.log 2>&1 || { tail $OUT/pmc.log; exit 3; }
tail -1 $OUT/pmc.log
cp $R/gpurun_out/${N}_pmc/pmc_traffic.json $R/profiles/${TAG}_pmc_traffic.json  # (this copy stays on the box)
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { tail $OUT/bench.log; exit 4; }
tail -1 $OUT/bench.log > $OUT/bench.json; cut -c1-300 $OUT/bench.json
timeout -k 10 200 python bench.py --shard-of 8 --no-cpu-baseline > $OUT/shard8.log 2>&1 || { tail $OUT/shard8.log; exit 5; }
tail -1 $OUT/shard8.log > $OUT/shard8.json
timeout -k 10 300 python bench.py --width 3840 --height 2160 --spp 8 --shard-of 8 --steps 10 --no-cpu-baseline > $OUT/c5_shard8.log 2>&1 || { tail $OUT/c5_shard8.log; exit 6; }
tail -1 $OUT/c5_shard8.log > $OUT/c5_shard8.json
timeout -k 10 200 python bench.py --scene flat --no-cpu-baseline > $OUT/flat.log 2>&1 || { tail $OUT/flat.log; exit 7; }
tail -1 $OUT/flat.log > $OUT/flat.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python $R/bench.py --steps 10 --no-cpu-baseline > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 8; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats.csv; head -8 $OUT/kernel_stats.csv | cut -c1-150
grep "^{\"metric\"" $OUT/prof.log | tail -1 > $OUT/prof_bench.json
# every frame with the shadow walks on the render stream (--overlap 0): each launch runs alone, as in
# bench's serialised roofline frames, so roofline.avg_launch_ms recomputes from this summary
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_serial -o run -- python $R/bench.py --steps 10 --overlap 0 --no-cpu-baseline > $OUT/prof_serial.log 2>&1 || { tail $OUT/prof_serial.log; exit 11; }
f=$(find $OUT/prof_serial -name "*kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats_serial.csv; head -8 $OUT/kernel_stats_serial.csv | cut -c1-150
grep "^{\"metric\"" $OUT/prof_serial.log | tail -1 > $OUT/prof_serial_bench.json
cd $R && bash tools/timeline.sh ${N}_tl > $OUT/tl.log 2>&1 || { tail $OUT/tl.log; exit 9; }
cp $R/gpurun_out/${N}_tl/n1.timeline $R/gpurun_out/${N}_tl/n8.timeline $OUT/ 2>/dev/null
timeout -k 10 200 python tools/phase_occupancy.py conference flat > $OUT/phases.jsonl 2>$OUT/phases.err || { tail $OUT/phases.err; exit 10; }
cut -c1-400 $OUT/phases.jsonl
echo final-done
