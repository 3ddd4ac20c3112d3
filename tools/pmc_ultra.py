"""Minimal driver for rocprofv3 passes over the UltraNet bench workload (b256 @416 fused forward): build the
network, run `--iters` forwards of a resident batch, nothing else (tools/profile_cmd_pmc.sh OUT tools/pmc_ultra.py)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--lib", default="", help="another build of the library (diagnostic variants)")
    a = ap.parse_args()
    from quantized_vit_amd import _lib
    from quantized_vit_amd.ultranet import random_ultranet, synthetic_images_u8
    if a.lib:
        _lib.load(a.lib)
    _lib.load()
    dev = torch.device("cuda", 0)
    model = random_ultranet(seed=0, device=dev)
    x = synthetic_images_u8(a.batch, 416, seed=1000, device=dev)
    with torch.no_grad():
        model(x)
        for _ in range(a.iters):
            model(x)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
