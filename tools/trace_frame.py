"""Prints the kernel timeline of the last frame in a rocprofv3 kernel trace (CSV or rocpd .db)."""
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
first = [i for i, r in enumerate(rows) if "k_raygen" in r[0]][-1]
t0 = rows[first][1]
for n, s, e, q in rows[first:]:
    print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{q} {n[:60]}")
