"""Prints the kernel timeline of the last product frame in a rocprofv3 kernel trace (CSV or rocpd
.db): frames start at k_raygen, at the level-1 packet walk that generates its rays, or, with level 1
fused, at k_trace_packet_shade; the last frame that
starts with the fused kernel is a timed frame of bench.py (its profiling frames after the timed
ones run level 1 unfused), else the last frame."""
import csv, sqlite3, sys


def rows_of(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
        name = "name" if "name" in cols else "kernel_name"
        q = f"select {name}, start, end, queue_id from kernels" if "queue_id" in cols else f"select {name}, start, end, 0 from kernels"
        return [(n, int(s), int(e), q) for n, s, e, q in c.execute(q)]
    return [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"])
            for r in csv.DictReader(open(path))]


rows = sorted(rows_of(sys.argv[1]), key=lambda r: r[1])
# (round 6: with level 1 unfused the packet walk generates the camera rays itself, tuning key 33, and
# starts the frame; after a k_raygen it does not)
starts = [i for i, r in enumerate(rows)
          if "k_raygen" in r[0] or ("k_trace_packet" in r[0] and not (i > 0 and "k_raygen" in rows[i - 1][0]))]
fused = [i for i in starts if "k_trace_packet_shade" in rows[i][0]]
first = fused[-1] if fused else starts[-1]
end = next((i for i in starts if i > first), len(rows))
t0 = rows[first][1]
for n, s, e, q in rows[first:end]:
    print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{q} {n[:60]}")
