"""Summarise rocprofv3 --pmc CSVs of tools/pmc_run.sh into bytes beyond L2 per launch per kernel.

usage: python tools/pmc_summary.py <pmc_run output dir> <out.json> [bench arguments of the profiled command]

FETCH_SIZE / WRITE_SIZE are in KiB.  Per /opt/skills/guides/MI355X_MICROARCH.md (HBM section)
FETCH_SIZE on gfx950 reads exactly half of the bytes of a wide (16 B/lane) stream, so the read
side is doubled; the kernels' loads are 12- and 16-byte gathers, near that regime.  Both
counters count memory-side (L2 -> fabric) traffic: Infinity-Cache hits are included, so this is
"bytes beyond L2", an upper bound on HBM bytes.  Other counters of the run (TCC hit rate, SQ and
TA / TD busy) are averaged per kernel as they are.
"""
import csv, glob, json, os, re, sys
from collections import defaultdict

# the kernels of the timed frames in the default (exact, cull mode 3) configuration, as bench.py's
# roofline names them: level 1's packet walk (k_trace_packet; k_trace_packet_shade where level 1 is
# fused, tuning key 17), the per-lane closest-hit walk of the deeper levels, the shadow walk and the
# lean PathTracer shading kernel
# (k_trace_packet<false, 3, kGen>: kGen, round 6, the walk generating its camera rays; k_shade<2, false,
# kRegen>: kRegen, level 1's shading regenerating them - both instantiations are the k_shade of levels 1-5)
PRODUCT = {"k_trace": (r"k_trace<false, 1, 3>",), "k_trace_packet_shade": (r"k_trace_packet_shade<2, 3>",),
           "k_trace_packet": (r"k_trace_packet<false, 3, ",),
           "k_shadow": (r"k_shadow<false, 1, 3>",), "k_shade": (r"k_shade<2, false, ",)}
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import kernel_source_stamp, workload_key  # noqa: E402


def profiled_workload(extra):
    """bench.py's workload key for the bench arguments of the profiled command."""
    import argparse
    p = argparse.ArgumentParser()
    for k, v in (("--width", 1920), ("--height", 1080), ("--spp", 4), ("--max-depth", 5), ("--shader", 2),
                 ("--shard-of", 0)):
        p.add_argument(k, type=int, default=v)
    p.add_argument("--scene", default="conference")
    a, _ = p.parse_known_args(extra)
    return workload_key(a, a.shard_of if a.shard_of > 1 else 0)


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
           "kernel_source_sha256": kernel_source_stamp(), "workload": profiled_workload(sys.argv[3:]),
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
