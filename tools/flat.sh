#!/bin/bash
# Flat-geometry stand-in rehearsal: PMC passes keyed to the flat workload, the
# phase occupancy of both stand-ins, and the flat bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd)
N=${1:-flat}; OUT=$R/gpurun_out/$N; mkdir -p $OUT
export PYTHONUNBUFFERED=1
python -c "from mobileraytracer_amd import _native as n; assert n.build_is_current(), 'stale libmobilert_amd.so'" || exit 2
timeout -k 10 200 python bench.py --scene flat --no-cpu-baseline > $OUT/flat.log 2>&1 || { tail $OUT/flat.log; exit 3; }
tail -1 $OUT/flat.log > $OUT/flat.json; cut -c1-300 $OUT/flat.json
timeout -k 10 300 python tools/phase_occupancy.py conference flat > $OUT/phases.jsonl 2>$OUT/phases.err || { tail $OUT/phases.err; exit 4; }
cut -c1-300 $OUT/phases.jsonl
bash tools/pmc_run.sh ${N}_pmc --scene flat > $OUT/pmc.log 2>&1 || { tail $OUT/pmc.log; exit 5; }
tail -3 $OUT/pmc.log
echo flat-done
