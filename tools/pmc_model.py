"""Minimal driver for rocprofv3 passes over the bench workload: build the quantized model, run
`--iters` forwards of a `--batch` resident batch, nothing else (no parity, no CPU baseline), so the
last dispatches of every hot kernel are exactly the profiled forwards (tools/pmc_model_summary.py).

    rocprofv3 --pmc ... --kernel-trace -d OUT -o run -- python tools/pmc_model.py [--model M --batch B]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="vit_base_patch16_224")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=2)
    a = ap.parse_args()
    from quantized_vit_amd import _lib
    from quantized_vit_amd.calibrate import VIT_CONFIGS, build_quantized_vit, synthetic_images
    _lib.load()
    dev = torch.device("cuda", 0)
    model = build_quantized_vit(a.model, seed=0, device=dev)
    x = synthetic_images(a.batch, VIT_CONFIGS[a.model]["img_size"], seed=1000, device=dev)
    with torch.no_grad():
        model(x)   # warm-up: plans, packed weights and code tables built here
        torch.cuda.synchronize()
        for _ in range(a.iters):
            model(x)
        torch.cuda.synchronize()
    print(f"pmc_model: {a.model} b{a.batch} x{a.iters} forwards done", flush=True)


if __name__ == "__main__":
    main()
