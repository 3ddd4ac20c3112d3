"""Times qvit_layernorm_quant_i8 on the ViT-B/16 b256 shape (50 432 x 768 fp32 rows -> int8 codes through
the quantizer's code table) with HIP events; reports the algorithmic HBM rate (row read + code write).

    python tools/ln_bench.py [--lib path] [--iters 50]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantized_vit_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rows", type=int, default=256 * 197)
    a = ap.parse_args()
    if a.lib:
        _lib.load(a.lib)
    from quantized_vit_amd.quant_layers import epilogue_table_geometry, saturation_level
    dev = torch.device("cuda:0")
    rows, cols = a.rows, 768
    x = torch.randn(rows, cols, device=dev) * 3.0
    gamma, beta = torch.rand(cols, device=dev) + 0.5, torch.randn(cols, device=dev) * 0.1
    qm, t = 3.0, 0.9
    d = qm ** t / 127
    pd, pqm, pt = (torch.tensor([v], device=dev) for v in (d, qm, t))
    geo = epilogue_table_geometry(_lib.QT_NONLINEAR, d, qm, t, saturation_level(_lib.QT_NONLINEAR, d, qm, t), False)
    table = _lib.epi_table_build(_lib.EPI_I8, _lib.QT_NONLINEAR, pd, pqm, pt, 0, *geo, dev)
    out = torch.empty(rows, cols, dtype=torch.int8, device=dev)
    fn = lambda: _lib.layernorm_quant_i8(x, gamma, beta, 1e-6, _lib.QT_NONLINEAR, pd, pqm, pt, 0, out, cols,
                                         code_table=table)
    ts = []
    for _ in range(a.iters + 5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        ts.append((s, e))
    torch.cuda.synchronize()
    ms = sorted(s.elapsed_time(e) for s, e in ts[5:])
    med = ms[len(ms) // 2]
    gbytes = rows * cols * 5 / 1e9
    print(f"layernorm+quant {rows}x{cols}: {med*1e3:.1f} us  {gbytes/med*1e3/1e3:.2f} TB/s algorithmic", flush=True)


if __name__ == "__main__":
    main()
