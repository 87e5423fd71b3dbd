"""BASELINE c3 as a workload: one ModelNet40 classify train step of the sph-dg
PVCNN_classifier mirror (PVCNN/models/pvcnn_classify.py:14-345 of the
reference; configs/modelnet40/pvcnn/experiments/SO3_SO3/exp13.py) on B
clouds of N points: forward (LRF change_coords, ball-query local PPF,
spherical voxelize / devoxelize, Conv3d blocks), cross-entropy loss,
backward (devoxelize / voxelize gradients) and an SGD step.  Synthetic
clouds (seeded gaussian, ModelNet40-like extent), random labels and
random-init weights; no dataset.

Prints one JSON line: ms per step, clouds/s, and the share of the step's
GPU time spent in this repository's kernels (pcr::) vs the torch / MIOpen
layers around them, from torch.profiler's device-side totals.

usage: python scripts/c3_train_step.py [--batch 256] [--points 2048] [--steps 5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
sys.path[:0] = [ROOT, PKG, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

# configs/modelnet40/pvcnn/__init__.py:5-8
DIM_K = 512
BLOCKS = ((64, 1, 32), (128, 1, 32), (256, 1, None), (DIM_K, 1, None))


def sph_dg():
    from PVCNN.models.pvcnn_classify import PVCNN_classifier
    return PVCNN_classifier(blocks=BLOCKS, dim_k=DIM_K, point_kernel_formal="dgcnn_kernel",
                            voxel_shape="spherical", num_classes=40, extra_feature_channels=0,
                            rot_invariant_preprocess="change_coords", with_local_feat="ppf",
                            with_transform_fine_tune=False, use_new_coords_for_voxel=False,
                            with_coeff=True, with_se=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--points", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    b, n = args.batch, args.points
    g = torch.Generator(device=dev).manual_seed(1)
    xyz = torch.randn((b, 3, n), generator=g, device=dev) * 0.35
    nrm = torch.randn((b, 3, n), generator=g, device=dev)
    nrm = nrm / nrm.norm(dim=1, keepdim=True)
    x = torch.cat([xyz, nrm], dim=1).contiguous()
    y = torch.randint(0, 40, (b,), generator=g, device=dev)
    model = sph_dg().to(dev).train()
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9)

    def step():
        opt.zero_grad(set_to_none=True)
        loss = torch.nn.functional.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / args.steps * 1e3

    # device time split: this repository's kernels vs everything else
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        step()
        torch.cuda.synchronize()
    ours, other, top = 0.0, 0.0, {}
    for e in prof.key_averages():
        t = e.device_time_total if hasattr(e, "device_time_total") else e.cuda_time_total
        if t <= 0 or e.key.startswith("aten::") or e.key.startswith("Memcpy"):
            continue
        if "pcr::" in e.key:
            ours += t
            short = e.key.split("(")[0].replace("void pcr::", "").split("<")[0]
            top[short] = top.get(short, 0.0) + t
        else:
            other += t
    print(json.dumps({
        "workload": "BASELINE c3: sph-dg PVCNN_classifier train step (forward, cross-entropy, "
                    "backward, SGD), synthetic clouds, random-init weights",
        "batch": b, "points": n, "steps": args.steps, "ms_per_step": round(ms, 3),
        "clouds_per_s": round(b / (ms * 1e-3), 1), "loss": float(loss),
        "device_ms_pcr_kernels": round(ours / 1e3, 3),
        "device_ms_other": round(other / 1e3, 3),
        "pcr_kernels_ms": {k: round(v / 1e3, 3) for k, v in
                           sorted(top.items(), key=lambda kv: -kv[1])},
    }))


if __name__ == "__main__":
    main()
