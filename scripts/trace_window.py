"""Diagnostic: print a window of a rocprofv3 kernel trace (start/end in us
relative to the window start, queue, kernel) around the middle of the run, and
per-kernel average durations.  Not part of the product."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
key = sys.argv[2] if len(sys.argv) > 2 else "select"
cnt = int(sys.argv[3]) if len(sys.argv) > 3 else 30
idx = [i for i, r in enumerate(rows) if key in r["Kernel_Name"]]
i0 = idx[len(idx) // 2]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i0 + cnt]:
    s = int(r["Start_Timestamp"]) - t0
    e = int(r["End_Timestamp"]) - t0
    print("%8.1f %8.1f %6.1f q%s %s" % (s / 1e3, e / 1e3, (e - s) / 1e3, r["Queue_Id"],
                                        r["Kernel_Name"][:60]))
d = collections.defaultdict(list)
for r in rows:
    d[r["Kernel_Name"][:60]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print("%5d x %8.2f us  %s" % (len(v), sum(v) / len(v) / 1e3, k))
