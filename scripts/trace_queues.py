"""Per-queue kernel timeline (start, duration, gap before) of a window of the
last runner call in a rocprofv3 kernel trace CSV.
usage: python scripts/trace_queues.py <kernel_trace.csv> [steps_per_call] [first] [count]"""
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "pcr::" not in n:
        continue
    short = n.split("(")[0].replace("void pcr::", "").split("<")[0]
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short, r["Queue_Id"]))
rows.sort()
per_call = int(sys.argv[2]) if len(sys.argv) > 2 else 80
first = int(sys.argv[3]) if len(sys.argv) > 3 else per_call // 2
count = int(sys.argv[4]) if len(sys.argv) > 4 else 6
st = [r for r in rows if r[2] == "vox_stream_kernel"][-per_call:]
t0, t1 = st[first][0], st[first + count][1]
byq = {}
for r in rows:
    if r[0] >= t0 and r[1] <= t1:
        byq.setdefault(r[3], []).append(r)
for q, lst in sorted(byq.items()):
    print("queue", q)
    prev = None
    for s, e, n, _ in lst:
        print("   %-26s start %8.1f dur %6.1f gap %6.1f" % (
            n, (s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3 if prev else 0))
        prev = e
