"""Per-stream busy time per step of the native runner's steady state, from a
rocprofv3 kernel trace CSV: the last runner call's steps minus 5 at each end.
usage: python scripts/stream_busy.py <kernel_trace.csv> [steps_per_call]"""
import csv
import sys
from collections import defaultdict

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "pcr::" not in n:
        continue
    short = n.split("(")[0].replace("void pcr::", "").split("<")[0]
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short, r["Queue_Id"]))
rows.sort()
per_call = int(sys.argv[2]) if len(sys.argv) > 2 else 40
st = [r for r in rows if r[2] in ("vox_stream_kernel", "vox_blocks_kernel")][-per_call:]
t0, t1 = st[5][0], st[-5][1]
win = [r for r in rows if r[0] >= t0 and r[1] <= t1]
nsteps = sum(1 for r in win if r[2] in ("vox_stream_kernel", "vox_blocks_kernel"))
print("steady steps %d, wall per step %.1f us" % (nsteps, (t1 - t0) / 1e3 / nsteps))
busy, kb, cnt = defaultdict(float), defaultdict(float), defaultdict(int)
for s, e, n, q in win:
    busy[q] += (e - s) / 1e3
    kb[(q, n)] += (e - s) / 1e3
    cnt[(q, n)] += 1
for q in sorted(busy):
    print("queue %s busy per step %.1f us" % (q, busy[q] / nsteps))
    for (qq, n), v in sorted(kb.items()):
        if qq == q:
            print("    %-24s %6.1f us/step (%d launches)" % (n, v / nsteps, cnt[(qq, n)]))
