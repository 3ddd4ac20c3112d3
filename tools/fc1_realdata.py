"""The fc1 GEMM on the model's own data: ViT-B/16 b256, block `--block`'s fc1 input codes captured from a
real forward, then the fc1 launch (W4, GELU + fc2 quantizer epilogue) timed alone with HIP events, and,
with a -DQVIT_GEMM_STAMPS --lib, its phase breakdown (tools/gemm_stamps.py phases).

    python tools/fc1_realdata.py [--block 5] [--lib tools/_diag/libqvit_hip_stamps.so --stamps]
"""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantized_vit_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--block", type=int, default=5)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--lib", default="")
    ap.add_argument("--stamps", action="store_true")
    a = ap.parse_args()
    lib = _lib.load(a.lib) if a.lib else _lib.load()
    from quantized_vit_amd import vit_model
    from quantized_vit_amd.calibrate import build_quantized_vit, synthetic_images
    from quantized_vit_amd.quant_layers import epilogue_table
    dev = torch.device("cuda:0")
    model = build_quantized_vit("vit_base_patch16_224", seed=0, device=dev)
    x = synthetic_images(256, 224, seed=1000, device=dev)
    fc1 = model.blocks[a.block].mlp.fc1
    fc2 = model.blocks[a.block].mlp.fc2
    cap = {}
    orig = fc1.gemm_codes

    def grab(codes, plan, epi, out=None, next_layer=None):
        cap["codes"] = codes.clone()
        return orig(codes, plan, epi, out=out, next_layer=next_layer)

    fc1.gemm_codes = grab
    with torch.no_grad():
        model(x)
    fc1.gemm_codes = orig
    codes = cap["codes"]
    p1, p2 = fc1.quant_plan(), fc2.quant_plan()
    hid = torch.empty((codes.shape[0], p2.kpad), dtype=torch.int8, device=dev)
    nz = (codes != 0).float().mean().item()
    print(f"block {a.block} fc1 input codes: M={codes.shape[0]} K={p1.kpad}, nonzero {nz:.3f}, "
          f"mean |code| {codes.float().abs().mean().item():.2f}", flush=True)
    if a.stamps:
        lib.qvit_gemm_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
        buf = (ctypes.c_ulonglong * 8)()
        torch.cuda.synchronize()
        assert lib.qvit_gemm_stamps(buf, 1) == 0
    ts = []
    for _ in range(a.iters + 3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fc1.gemm_codes(codes, p1, _lib.EPI_I8_GELU, out=hid, next_layer=fc2)
        e.record()
        ts.append((s, e))
    torch.cuda.synchronize()
    ms = sorted(s.elapsed_time(e) for s, e in ts[3:])
    med = ms[len(ms) // 2]
    ops = 2.0 * codes.shape[0] * p1.n * p1.kpad
    print(f"fc1 real data: {med*1e3:.1f} us  {ops/med/1e9:.1f} TOPS  {ops/med/1e9/5033.16*100:.1f}% of int8 peak",
          flush=True)
    if a.stamps:
        assert lib.qvit_gemm_stamps(buf, 0) == 0
        waves = max(buf[7], 1)
        names = ["head_wait", "dma_issue", "stage_wait", "reads+mfma", "epilogue", "tile_setup", "lgkm_wait"]
        per = [buf[i] / waves for i in range(7)]
        tot = sum(per)
        print("per wave: " + "  ".join(f"{n} {v:8.0f} ({100*v/tot:4.1f}%)" for n, v in zip(names, per)))
    del vit_model, epilogue_table


if __name__ == "__main__":
    main()
