"""Lists the device operations of ONE warm bench step (ViT-B/16 b256 by default) with torch.profiler:
every kernel and memcpy/memset with its count and total device time, so launches that are not hot
kernels (copies, fills, small torch ops) show up with their share of the step.

    python tools/step_ops.py [--batch 256] [--model vit_base_patch16_224]
"""
import argparse
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantized_vit_amd.calibrate import build_quantized_vit, synthetic_images  # noqa: E402
from quantized_vit_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--model", default="vit_base_patch16_224")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    _lib.load()
    model = build_quantized_vit(args.model, seed=0, device=dev)
    x = synthetic_images(args.batch, 224 if "224" in args.model else 384, seed=1000, device=dev)
    with torch.no_grad():
        for _ in range(3):
            model(x)
        torch.cuda.synchronize()
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            model(x)
            torch.cuda.synchronize()
    agg = defaultdict(lambda: [0, 0.0])
    for e in prof.events():
        if e.device_type == torch.autograd.DeviceType.CUDA:
            a = agg[e.name[:90]]
            a[0] += 1
            a[1] += e.device_time_total if hasattr(e, "device_time_total") else e.cuda_time_total
    tot = sum(v[1] for v in agg.values())
    print(f"device ops in one step: {sum(v[0] for v in agg.values())}, {tot / 1e3:.3f} ms")
    for name, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{n:5d} {us:10.1f} us {100 * us / tot:5.1f}%  {name}")
    # the CPU-side ops that issued copies / fills: the aten callers
    print("\naten ops (CPU) with their counts:")
    ka = prof.key_averages()
    for k in sorted(ka, key=lambda k: -k.count)[:40]:
        if k.key.startswith("aten::"):
            print(f"{k.count:5d}  {k.key}")


if __name__ == "__main__":
    main()
