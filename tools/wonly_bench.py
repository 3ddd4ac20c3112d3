"""Weight-only QuantizeLinear: qvit_gemm_wonly against the reference's arithmetic on the library path
(F.linear on the fp32 fake-quant weight, hipBLASLt), ViT-B/16 layer shapes at batch 256 and batch 1.

    python tools/wonly_bench.py [--iters 20] [--json out.json]

Times each launch with HIP events on the launch stream (median). TFLOP/s counts 2 M N K (the layer's own
flops, not the three bf16 passes).
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from quantized_vit_amd import _lib  # noqa: E402

SHAPES = {"qkv": (2304, 768), "proj": (768, 768), "fc1": (3072, 768), "fc2": (768, 3072)}


def timed(fn, iters):
    ts = []
    for _ in range(iters + 3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    ts = sorted(ts[3:])
    return ts[len(ts) // 2] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    from test_gpu_kernels import pack_codes
    rows = []
    for M in (256 * 197, 197):
        for name, (N, K) in SHAPES.items():
            g = torch.Generator().manual_seed(N + K)
            codes = torch.randint(-8, 8, (N, K), generator=g)
            packed, npad, kpad = pack_codes(codes, _lib.W4, dev)
            d_w = torch.tensor([0.01], device=dev)
            bias = torch.randn(N, generator=g).to(dev)
            bias_pad = _lib.pad_bias(bias, N, npad, dev)
            x = torch.randn(M, K, generator=g).to(dev)
            y = torch.empty((M, N), device=dev)
            wq = (0.01 * codes.float()).to(dev)
            us_k = timed(lambda: _lib.gemm_wonly(x, M, kpad, packed, _lib.W4, N, npad, d_w, bias_pad, y), a.iters)
            us_l = timed(lambda: F.linear(x, wq, bias), a.iters)
            err = ((y - F.linear(x.double(), wq.double(), bias.double()).float()).abs().max()
                   / F.linear(x.abs().double(), wq.abs().double(), bias.abs().double()).max()).item()
            tf = 2.0 * M * N * K / 1e12
            r = dict(layer=name, M=M, N=N, K=K, wonly_us=us_k, library_fp32_us=us_l, wonly_tflops=tf / (us_k * 1e-6),
                     library_tflops=tf / (us_l * 1e-6), speedup=us_l / us_k, max_rel_err=err)
            rows.append(r)
            print(f"{name:5s} M={M:6d} N={N:5d} K={K:5d}  wonly {us_k:8.1f} us ({r['wonly_tflops']:6.1f} TF/s)  "
                  f"F.linear fp32 {us_l:8.1f} us ({r['library_tflops']:6.1f} TF/s)  x{r['speedup']:.2f}  "
                  f"rel err {err:.2e}", flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
