"""Summarise rocprofv3 --pmc CSVs of tools/pmc_run.sh into bytes beyond L2 per launch per kernel.

usage: python tools/pmc_summary.py <pmc_run output dir> <out.json>

FETCH_SIZE / WRITE_SIZE are in KiB.  Per /opt/skills/guides/MI355X_MICROARCH.md (HBM section)
FETCH_SIZE on gfx950 reads exactly half of the bytes of a wide (16 B/lane) stream, so the read
side is doubled; the kernels' loads are 12- and 16-byte gathers, near that regime.  Both
counters count memory-side (L2 -> fabric) traffic: Infinity-Cache hits are included, so this is
"bytes beyond L2", an upper bound on HBM bytes.  Other counters of the run (TCC hit rate, SQ and
TA / TD busy) are averaged per kernel as they are.
"""
import csv, glob, json, os, re, sys
from collections import defaultdict

# the default (exact, cull mode 3) walk instantiations and the lean PathTracer shading kernel;
# "k_trace" is every closest-hit launch of a frame: the camera rays' packet walk and the per-lane
# walk of the other levels, averaged over their dispatches as bench.py averages its launches
PRODUCT = {"k_trace": (r"k_trace<false, 1, 3>", r"k_trace_packet<false, 3>"), "k_shadow": (r"k_shadow<false, 1, 3>",),
           "k_shade": (r"k_shade<2, false>",)}
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import kernel_source_stamp  # noqa: E402


def rows(d):
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            yield from csv.DictReader(f)


def main():
    src, dst = sys.argv[1], sys.argv[2]
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> values (one per dispatch)
    for row in rows(src):
        per[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {"bytes_beyond_l2_per_launch": {}, "counters": {}, "kernels": {},
           "kernel_source_sha256": kernel_source_stamp(),
           "note": "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, KiB -> bytes, averaged over the dispatches of "
                   "the profiled command; includes Infinity-Cache hits"}
    for short, pats in PRODUCT.items():
        names = [k for k in per if any(p in k for p in pats)]
        if not names:
            continue
        c = defaultdict(list)  # counter -> values of every dispatch of these kernels
        for n in names:
            for k, v in per[n].items():
                c[k].extend(v)
        avg = {k: sum(v) / len(v) for k, v in c.items() if v}
        out["counters"][short] = avg
        out["kernels"][short] = names
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            out["bytes_beyond_l2_per_launch"][short] = (2.0 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024.0
        if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
            out["counters"][short]["l2_hit_rate"] = avg["TCC_HIT_sum"] / max(1.0, avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out["bytes_beyond_l2_per_launch"]))


main()
