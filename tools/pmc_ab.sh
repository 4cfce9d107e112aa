#!/bin/bash
# A/B of memory-pipeline PMC counters on the closest-hit trace kernel for trace variants
# (MRT_TRACE_VARIANT), one counter group per rocprofv3 run.  usage: pmc_ab.sh OUT V1 V2 ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${1:-pmc_ab}; shift; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  i=0
  for grp in "GRBM_GUI_ACTIVE TA_TA_BUSY TD_TD_BUSY" "TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES" \
             "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS"; do
    i=$((i+1))
    MRT_TRACE_VARIANT=$v timeout -k 10 240 rocprofv3 --pmc $grp --kernel-include-regex "k_trace<false" --output-format csv -d $OUT/v$v/p$i -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/v$v.p$i.log 2>&1 || { rc=$?; echo "pmc v$v pass $i failed rc=$rc"; tail -3 $OUT/v$v.p$i.log; exit $rc; }
  done
done
python3 - "$OUT" "$@" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for v in sys.argv[2:]:
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{out}/v{v}/p*/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
    avg = {k: sum(x) / len(x) for k, x in acc.items()}
    print(f"variant {v}: " + "  ".join(f"{k}={avg[k]:.4g}" for k in sorted(avg)))
PY
