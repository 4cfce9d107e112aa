"""Summarise rocprofv3 --pmc CSVs (FETCH_SIZE / WRITE_SIZE passes) for the trace kernel.

usage: python tools/pmc_summary.py <fetch_counter_collection.csv> <write_counter_collection.csv> <out.json>

FETCH_SIZE / WRITE_SIZE are in KiB.  Per /opt/skills/guides/MI355X_MICROARCH.md (HBM section) FETCH_SIZE
on gfx950 reads exactly half of the bytes of a wide (16 B/lane) coalesced stream, so the read side
is doubled; the trace kernel's loads are 16-byte (float4) gathers, the regime the correction was
measured in.  Both counters count memory-side (L2 -> fabric) traffic: Infinity-Cache hits are
included, so this is "bytes beyond L2", an upper bound on HBM bytes.
"""
import csv, json, sys
from collections import defaultdict

def load(path, counter):
    per = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            per[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return per

fetch = load(sys.argv[1], "FETCH_SIZE")
write = load(sys.argv[2], "WRITE_SIZE")
out = {"kernels": {}}
for k in sorted(set(fetch) | set(write)):
    f = fetch.get(k, []); w = write.get(k, [])
    if not f:
        continue
    fk = sum(f) / len(f); wk = (sum(w) / len(w)) if w else 0.0
    out["kernels"][k] = {"launches": len(f), "fetch_kib_avg": fk, "write_kib_avg": wk,
                         "hbm_bytes_per_launch": (2.0 * fk + wk) * 1024.0}
trace = [k for k in out["kernels"] if "k_trace<false" in k]
if trace:
    out["trace_kernel"] = trace[0]
    out["hbm_bytes_per_launch"] = out["kernels"][trace[0]]["hbm_bytes_per_launch"]
out["note"] = "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, KiB -> bytes; includes Infinity-Cache hits"
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if k != "kernels"}))
