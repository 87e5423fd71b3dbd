"""Per-step timeline of the native runner from a rocprofv3 kernel trace CSV:
for a window of steady-state steps prints each kernel's start/end relative
to the window start (us), its stream and duration, and the gaps on each
stream.  usage: python scripts/trace_steps.py <kernel_trace.csv> [first] [count]"""
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "pcr::" not in n:
        continue
    short = n.split("(")[0].replace("void pcr::", "").split("<")[0]
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short, r["Queue_Id"],
                 r["LDS_Block_Size"], r["Grid_Size_X"], r["Grid_Size_Y"], r["Workgroup_Size_X"]))
rows.sort()
first = int(sys.argv[2]) if len(sys.argv) > 2 else len(rows) // 2
count = int(sys.argv[3]) if len(sys.argv) > 3 else 18
win = rows[first:first + count]
t0 = win[0][0]
for s, e, name, q, lds, gx, gy, wg in win:
    print("%-22s q%-2s start %8.1f end %8.1f dur %6.1f  lds %6s grid %sx%s wg %s"
          % (name, q, (s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, lds, gx, gy, wg))
