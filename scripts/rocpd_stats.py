"""Per-kernel duration summary (calls, average, min, max in us) from a
rocprofv3 SQLite output (rocpd *.db), for runs made without --output-format
csv.  usage: python scripts/rocpd_stats.py <dir-or-db> [name-filter]"""
import glob
import os
import sqlite3
import sys

path = sys.argv[1]
db = path if path.endswith(".db") else glob.glob(os.path.join(path, "**", "*.db"), recursive=True)[0]
flt = sys.argv[2] if len(sys.argv) > 2 else "pcr::"
con = sqlite3.connect(db)
cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
name_col = "name" if "name" in cols else "kernel_name"
rows = con.execute("select %s, start, end from kernels" % name_col).fetchall()
agg = {}
for name, s, e in rows:
    if flt not in name:
        continue
    short = name.split("(")[0].replace("void ", "")
    agg.setdefault(short, []).append((e - s) / 1000.0)
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print("%-70s %5d calls  avg %8.2f us  min %8.2f  max %8.2f" % (k[:70], len(v), sum(v) / len(v),
                                                                     min(v), max(v)))
