"""Diagnostic: from a rocprofv3 kernel trace, per-iteration start/end of the
KNN selection and the grid-streaming kernel (relative to the earlier start)
to see how they overlap.  Not part of the product."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
keys = sys.argv[2].split(",")
sel = [r for r in rows if any(k in r["Kernel_Name"] for k in keys)]
sel = sel[len(sel) // 2: len(sel) // 2 + int(sys.argv[3]) if len(sys.argv) > 3 else 24]
t0 = int(sel[0]["Start_Timestamp"])
for r in sel:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    e = (int(r["End_Timestamp"]) - t0) / 1e3
    print("%8.1f %8.1f %6.1f %s" % (s, e, e - s, r["Kernel_Name"][:50]))
