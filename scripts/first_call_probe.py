"""Why is bench.py's one timed 20-step call slower than the same call
repeated?  Replays bench.py main()'s order (workload, timing events,
verify, W warm-up steps, the timed call) and then repeats warm-up + timed
call TRIALS times; prints each trial's wall time.  PRE: untimed steps run
before the first warm-up (after verify).
usage: [TRIALS=6] [PRE=0] [PRE_CALL=0] [PRE_SLEEP=0] python scripts/first_call_probe.py [bench args]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

TRIALS = int(os.environ.get("TRIALS", "6"))
PRE = int(os.environ.get("PRE", "0"))
PRE_CALL = int(os.environ.get("PRE_CALL", "0"))  # steps per pre call (0: bench's chunking)
PRE_SLEEP = float(os.environ.get("PRE_SLEEP", "0"))  # host sleep (s) after the pre phase
args = bench.parse(sys.argv[1:] or ["--steps", "20", "--warmup", "5"])
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
t_start = time.perf_counter()
wl = bench.WORKLOADS[args.workload](args, dev, 0, 1)
wl.prepare_timing()
tv = time.perf_counter()
if not args.no_verify:
    wl.verify()
torch.cuda.synchronize()
print("setup %.1f ms, verify %.1f ms" % ((tv - t_start) * 1e3, (time.perf_counter() - tv) * 1e3),
      flush=True)
if PRE:
    t0 = time.perf_counter()
    if PRE_CALL:
        for _ in range(PRE // PRE_CALL):
            wl.run(PRE_CALL, timed=False)
            torch.cuda.synchronize()
    else:
        wl.run(PRE, timed=False)
    torch.cuda.synchronize()
    print("pre %d steps %.2f ms" % (PRE, (time.perf_counter() - t0) * 1e3), flush=True)
if PRE_SLEEP:
    time.sleep(PRE_SLEEP)
for trial in range(TRIALS):
    wl.run(args.warmup, timed=False)
    torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    wl.run(args.steps, timed=True)
    torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    ms = wl.ex.grid_kernel_times() if hasattr(wl, "ex") else []
    print("trial %d: %.3f ms = %.1f clouds/s, grid launches %s" % (
        trial, el * 1e3, args.batch * args.steps / el, " ".join("%.1f" % (m * 1e3) for m in ms)),
        flush=True)
