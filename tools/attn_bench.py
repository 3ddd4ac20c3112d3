"""Times qvit_attention on the ViT-B/16 b256 shape (B=256, N=197, H=12, hd=64) against torch's fp32
bmm + softmax + bmm sequence on the same qkv, with HIP events (median over iters)."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantized_vit_amd import _lib  # noqa: E402


def timeit(fn, iters):
    ts = []
    for _ in range(iters + 2):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        ts.append((s, e))
    torch.cuda.synchronize()
    ms = sorted(s.elapsed_time(e) for s, e in ts[2:])
    return ms[len(ms) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--N", type=int, default=197)
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--lib", default="", help="load this library build instead (diagnostic variants)")
    ap.add_argument("--split-only", action="store_true")
    ap.add_argument("--fused", action="store_true", help="also time qvit_qkv_attention (+ the qkv split GEMM)")
    ap.add_argument("--stamps", action="store_true", help="with a -DQVIT_ATT_STAMPS --lib: phase cycles")
    ap.add_argument("--w8", action="store_true", help="fused kernel on the int8 image (a diagnostic --lib)")
    a = ap.parse_args()
    if a.lib:
        _lib.load(a.lib)
    dev = torch.device("cuda:0")
    B, N, H = a.B, a.N, a.H
    qkv = torch.randn(B * N, 3 * H * 64, device=dev)
    out = torch.empty(B * N, H * 64, device=dev)
    codes = torch.empty(B * N, H * 64, dtype=torch.int8, device=dev)
    d, qm = torch.tensor([2.0 / 127], device=dev), torch.tensor([2.0], device=dev)
    t = torch.tensor([1.0], device=dev)

    def torch_ref():
        x = qkv.reshape(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
        at = ((x[0] @ x[1].transpose(-2, -1)) * 0.125).softmax(dim=-1)
        return (at @ x[2]).transpose(1, 2).reshape(B * N, H * 64)

    hi = qkv.half().reshape(-1)
    lo = (qkv - qkv.half().float()).half().reshape(-1)
    from quantized_vit_amd.quant_layers import epilogue_table_geometry, saturation_level
    geo = epilogue_table_geometry(_lib.QT_NONLINEAR, 2.0 / 127, 2.0, 1.0,
                                  saturation_level(_lib.QT_NONLINEAR, 2.0 / 127, 2.0, 1.0), False)
    table = _lib.epi_table_build(_lib.EPI_I8, _lib.QT_NONLINEAR, d, qm, t, 0, *geo, dev)   # as the model does
    sp = timeit(lambda: _lib.attention_split(hi, lo, B, N, H, 64, 0.125, codes, _lib.ATT_I8, 1.0, _lib.QT_NONLINEAR,
                                             d, qm, t, epi_table=table), a.iters)
    spf = timeit(lambda: _lib.attention_split(hi, lo, B, N, H, 64, 0.125, out), a.iters)
    flops = 4.0 * B * H * N * N * 64
    print(f"{'split i8':20s} {sp*1e3:9.1f} us  {flops/sp/1e9:8.1f} TFLOP/s (fp32-equivalent)", flush=True)
    print(f"{'split f32':20s} {spf*1e3:9.1f} us  {flops/spf/1e9:8.1f} TFLOP/s (fp32-equivalent)", flush=True)
    if a.stamps:
        import ctypes
        lib = _lib.load()
        lib.qvit_att_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
        buf = (ctypes.c_ulonglong * 16)()
        torch.cuda.synchronize()
        assert lib.qvit_att_stamps(buf, 1) == 0
        _lib.attention_split(hi, lo, B, N, H, 64, 0.125, codes, _lib.ATT_I8, 1.0, _lib.QT_NONLINEAR, d, qm, t,
                             epi_table=table)
        torch.cuda.synchronize()
        assert lib.qvit_att_stamps(buf, 0) == 0
        waves = max(buf[15], 1)
        per = [buf[i] / waves for i in range(6)]
        names = ["wait+issue", "scores", "softmax", "PV", "epilogue", "q-reads"]
        tot = sum(per)
        print("per wave: " + "  ".join(f"{n} {v:8.0f} ({100*v/tot:4.1f}%)" for n, v in zip(names, per)))
    if a.fused:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from test_gpu_kernels import act_buffer, pack_codes
        g = torch.Generator().manual_seed(1)
        C = 64 * H
        acodes = torch.randint(-60, 61, (B * N, 768), generator=g)
        w = torch.randint(-7, 8, (3 * C, 768), generator=g)
        packed, npad, kpad = pack_codes(w, _lib.W4, dev)
        packed8, _, _ = pack_codes(w, _lib.W8, dev)
        bias_pad = _lib.pad_bias((torch.randn(3 * C, generator=g) * 0.3).to(dev), 3 * C, npad, dev)
        A = act_buffer(acodes, kpad, dev)
        da, dw = torch.tensor([0.004], device=dev), torch.tensor([0.003], device=dev)
        wimg, wf = (packed8, _lib.W8) if a.w8 else (packed, _lib.W4)
        fz = lambda: _lib.qkv_attention(A, B, N, kpad, wimg, npad, da, dw, bias_pad, H, 0.125, codes, _lib.ATT_I8,
                                        1.0, _lib.QT_NONLINEAR, d, qm, t, epi_table=table, wfmt=wf)
        ms = timeit(fz, a.iters)
        print(f"{'fused qkv+attn i8':20s} {ms*1e3:9.1f} us", flush=True)
        outf = torch.empty(B * N, C, device=dev)
        ms = timeit(lambda: _lib.qkv_attention(A, B, N, kpad, wimg, npad, da, dw, bias_pad, H, 0.125, outf,
                                               _lib.ATT_F32, 1.0, wfmt=wf), a.iters)
        print(f"{'fused qkv+attn f32':20s} {ms*1e3:9.1f} us", flush=True)
        hi2 = torch.empty(B * N * 3 * C, dtype=torch.float16, device=dev)
        lo2 = torch.empty_like(hi2)
        ms2 = timeit(lambda: _lib.gemm_qkv_split(A, B * N, kpad, packed, _lib.W4, 3 * C, npad, da, dw, bias_pad, N, 1.0,
                                                 hi2, lo2), a.iters)
        print(f"{'qkv split gemm':20s} {ms2*1e3:9.1f} us", flush=True)
        if a.stamps:
            import ctypes
            lib = _lib.load()
            lib.qvit_qkv_att_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
            buf = (ctypes.c_ulonglong * 16)()
            torch.cuda.synchronize()
            assert lib.qvit_qkv_att_stamps(buf, 1) == 0
            fz()
            torch.cuda.synchronize()
            assert lib.qvit_qkv_att_stamps(buf, 0) == 0
            waves = max(buf[15], 1)
            per = [buf[i] / waves for i in range(10)]
            names = ["attn tail", "scores", "softmax", "PV", "store", "load issue", "w write(wait)", "barrier",
                     "proj reads+mfma", "proj epilogue"]
            tot = sum(per)
            print("fused per wave: " + "  ".join(f"{n} {v:8.0f} ({100*v/tot:4.1f}%)" for n, v in zip(names, per)))
    if a.split_only:
        return
    f32 = timeit(lambda: _lib.attention(qkv, B, N, H, 64, 0.125, out), a.iters)
    i8 = timeit(lambda: _lib.attention(qkv, B, N, H, 64, 0.125, codes, _lib.ATT_I8, 1.0, _lib.QT_NONLINEAR, d, qm, t),
                a.iters)
    tr = timeit(torch_ref, a.iters)
    for name, ms in (("qvit_attention f32", f32), ("qvit_attention i8", i8), ("torch fp32", tr)):
        print(f"{name:20s} {ms*1e3:9.1f} us  {flops/ms/1e9:8.1f} TFLOP/s (fp32-equivalent)", flush=True)


if __name__ == "__main__":
    main()
