#!/bin/bash
# Instruction-mix PMC passes over the trace kernels (packet walk vs per-lane walk).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${1:-ppmc}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
CMD="python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline"
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" "SQ_INST_CYCLES_SALU SQ_INST_CYCLES_SMEM SQ_INST_LEVEL_SMEM SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "k_trace" --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1 || { rc=$?; echo "pass $i failed rc=$rc"; tail -5 $OUT/p$i.log; exit $rc; }
done
python - $OUT <<'PY'
import csv, glob, os, sys
from collections import defaultdict
per = defaultdict(lambda: defaultdict(list))
for p in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(p)):
        per[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in per.items():
    print(k[:60])
    for n, v in sorted(c.items()):
        print("   %-22s %14.4g (n=%d)" % (n, sum(v) / len(v), len(v)))
PY
