"""UltraNet 4-bit forward throughput (BASELINE configs[4]): fused HIP path, synthetic k/255 416x416
images, random-init calibrated network. Reports img/s, int8 TOPS (2 x 674.4 M MAC/img) and the
algorithmic HBM rate (image fp32 in + every layer's codes written and read once + head/decode out).

    python tools/ultranet_bench.py [--batch 64] [--steps 20] [--warmup 5]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantized_vit_amd.ultranet import random_ultranet, synthetic_images_u8  # noqa: E402

MAC_PER_IMG = 674.4e6


def algorithmic_bytes_per_img(size=416):
    s = size
    b = 3 * s * s * 4                      # fp32 image
    acts = [(s // 2) ** 2 * 16, (s // 4) ** 2 * 32, (s // 8) ** 2 * 64, (s // 16) ** 2 * 64] + [(s // 16) ** 2 * 64] * 4
    b += 2 * sum(acts)                     # each layer's codes written once, read once
    g = (s // 16) ** 2
    b += g * 36 * 4 * 2                    # head fp32 out + decode read
    b += 2 * g * 36 * 4                    # io + p
    return b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--lib", default="", help="time another build of the library (same-box A/B)")
    a = ap.parse_args()
    if a.lib:
        from quantized_vit_amd import _lib
        _lib.load(a.lib)
    dev = torch.device("cuda:0")
    model = random_ultranet(seed=0, device=dev)
    x = synthetic_images_u8(a.batch, 416, seed=1, device=dev)
    with torch.no_grad():
        assert model.fused_ok(x)
        for _ in range(a.warmup):
            model(x)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.steps):
            model(x)
        e.record()
        torch.cuda.synchronize()
    ms = s.elapsed_time(e) / a.steps
    ips = a.batch / (ms * 1e-3)
    res = {"workload": f"UltraNetQua W4A4 fused forward, batch {a.batch}, 416x416", "ms_per_step": ms, "img_per_s": ips,
           "tops": 2 * MAC_PER_IMG * ips / 1e12, "algorithmic_GBps": algorithmic_bytes_per_img() * ips / 1e9}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
