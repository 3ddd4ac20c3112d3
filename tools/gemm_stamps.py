"""Where a GEMM wave's cycles go: runs the GEMM microbenchmark shapes on a diagnostic build of the
library (-DQVIT_GEMM_STAMPS: s_memtime stamps around each pipeline phase, summed over waves) and
prints the per-wave phase breakdown in shader cycles.

    python tools/gemm_stamps.py --build          # here (no GPU): compile tools/_diag/libqvit_hip_stamps.so
    python tools/gemm_stamps.py [--shapes fc1_i32,fc2]   # on the GPU box

Phases of the persistent kernel, summed over a wave's tiles: tile head (stage-0 wait), DMA issue,
stage wait (vmcnt + barrier), fragment reads + MFMA issue (incl. the two tail steps), epilogue, and
tile setup (next-tile sources, accumulator reset). Stamps cost cycles themselves;
compare phases within one run, not against the product library's wall time.
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
DIAG = os.path.join(ROOT, "tools", "_diag")
LIB = os.path.join(DIAG, "libqvit_hip_stamps.so")
PHASES = ["head_wait", "dma_issue", "stage_wait", "reads+mfma", "epilogue", "tile_setup", "ln_job"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--shapes", default="fc1_i32,fc1,qkv,fc2")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--lib", default="", help="another -DQVIT_GEMM_STAMPS build (path) instead of the default one")
    ap.add_argument("--build-var", nargs="*", default=[],
                    help="NAME=DEF1,DEF2 ...: build tools/_diag/libqvit_hip_NAME.so with those defines")
    ap.add_argument("--bench-var", default="", help="time variant library NAME (see --build-var)")
    ap.add_argument("--ws", default="", help="a -DQVIT_GEMM_WS_STAMPS build (path): the weight-stationary kernel's "
                    "per-tile k-loop / epilogue cycles, weight fill and clock")
    ap.add_argument("--light", default="", help="a -DQVIT_GEMM_LSTAMPS build (path): per-tile head / main loop / "
                    "epilogue cycles and the in-kernel clock")
    a = ap.parse_args()
    if a.light:
        light(a)
        return
    if a.ws:
        ws(a)
        return
    from quantized_vit_amd import build
    if a.build_var:
        for spec in a.build_var:
            name, defs = spec.split("=", 1)
            print(build.build(defines=tuple(d for d in defs.split(",") if d),
                              lib=os.path.join(DIAG, f"libqvit_hip_{name}.so"),
                              build_dir=os.path.join(DIAG, f"obj_{name}")))
        return
    if a.build:
        print(build.build(defines=("QVIT_GEMM_STAMPS",), lib=LIB, build_dir=os.path.join(DIAG, "obj")))
        return
    if a.bench_var:
        import torch
        from quantized_vit_amd import _lib
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import gemm_bench
        tag = a.bench_var
        _lib.load(os.path.join(DIAG, f"libqvit_hip_{tag}.so"))
        for name in a.shapes.split(","):
            M, N, K, epi = gemm_bench.SHAPES[name]
            r = gemm_bench.run(name, M, N, K, epi, 20, torch.device("cuda:0"))
            print(f"{tag} {name:8s} {r['ms']*1e3:8.1f} us  {100*r['frac']:5.1f}% of int8 peak", flush=True)
        return
    import torch
    from quantized_vit_amd import _lib
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gemm_bench
    lib = _lib.load(a.lib or LIB)
    lib.qvit_gemm_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.qvit_gemm_stamps.restype = ctypes.c_int
    dev = torch.device("cuda:0")
    buf = (ctypes.c_ulonglong * 8)()
    for name in a.shapes.split(","):
        M, N, K, epi = gemm_bench.SHAPES[name]
        torch.cuda.synchronize()
        assert lib.qvit_gemm_stamps(buf, 1) == 0
        r = gemm_bench.run(name, M, N, K, epi, a.iters, dev)
        torch.cuda.synchronize()
        assert lib.qvit_gemm_stamps(buf, 0) == 0
        waves = max(buf[7], 1)
        per = [buf[i] / waves for i in range(7)]
        tot = sum(per)
        nk = K // 64
        tiles = ((N + 255) // 256) * ((M + 127) // 128)
        blocks = min(tiles + (-tiles) % 8, torch.cuda.get_device_properties(0).multi_processor_count * 2)
        mfma_cyc = int(32 * nk * 16 * tiles / blocks)  # 32 MFMAs of 16 cycles per stage, per wave
        print(f"{name:8s} {r['ms']*1e3:7.1f} us  cycles/wave {tot:9.0f}  (MFMA floor {mfma_cyc})  " +
              "  ".join(f"{p} {v:7.0f} ({100*v/tot:4.1f}%)" for p, v in zip(PHASES, per)), flush=True)


def light(a):
    """Per-tile phase cycles from a light-stamp build: three s_memtime stamps per tile (no per-stage stamp, so the
    main loop runs as in the product), and the in-kernel clock from s_memtime / s_memrealtime (100 MHz)."""
    import torch
    from quantized_vit_amd import _lib
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gemm_bench
    lib = _lib.load(a.light)
    lib.qvit_gemm_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.qvit_gemm_stamps.restype = ctypes.c_int
    dev = torch.device("cuda:0")
    buf = (ctypes.c_ulonglong * 8)()
    for name in a.shapes.split(","):
        M, N, K, epi = gemm_bench.SHAPES[name]
        gemm_bench.run(name, M, N, K, epi, 3, dev)  # warm
        torch.cuda.synchronize()
        assert lib.qvit_gemm_stamps(buf, 1) == 0
        r = gemm_bench.run(name, M, N, K, epi, a.iters, dev)
        torch.cuda.synchronize()
        assert lib.qvit_gemm_stamps(buf, 0) == 0
        tiles = max(buf[5], 1)
        nk = K // 64
        floor = 32 * nk * 16  # one wave's MFMA cycles per tile (16 per 16x16x64 MFMA, 32 per stage)
        clk = buf[3] / max(buf[4], 1) * 0.1
        print(f"{name:8s} {r['ms']*1e3:7.1f} us  clock {clk:5.2f} GHz  per tile and wave: head {buf[0]/tiles:7.0f}  "
              f"main loop {buf[1]/tiles:7.0f} (MFMA alone {floor})  epilogue {buf[2]/tiles:7.0f}  "
              f"tiles/wave {tiles/max(buf[7],1):5.2f}  wave life {buf[3]/max(buf[7],1):9.0f} cyc", flush=True)


def ws(a):
    import torch
    from quantized_vit_amd import _lib
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gemm_bench
    lib = _lib.load(a.ws)
    lib.qvit_gemm_ws_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.qvit_gemm_ws_stamps.restype = ctypes.c_int
    dev = torch.device("cuda:0")
    buf = (ctypes.c_ulonglong * 8)()
    for name in a.shapes.split(","):
        M, N, K, epi = gemm_bench.SHAPES[name]
        gemm_bench.run(name, M, N, K, epi, 3, dev)
        torch.cuda.synchronize()
        assert lib.qvit_gemm_ws_stamps(buf, 1) == 0
        r = gemm_bench.run(name, M, N, K, epi, a.iters, dev)
        torch.cuda.synchronize()
        assert lib.qvit_gemm_ws_stamps(buf, 0) == 0
        tiles, waves = max(buf[5], 1), max(buf[7], 1)
        floor = (K // 32) * 6 * 32  # one wave's 32x32x32 MFMA cycles per 64 x 96 tile
        clk = buf[3] / max(buf[4], 1) * 0.1
        print(f"{name:8s} {r['ms']*1e3:7.1f} us  clock {clk:5.2f} GHz  per tile and wave: k-loop {buf[0]/tiles:7.0f} "
              f"(MFMA alone {floor})  epilogue {buf[1]/tiles:7.0f}  fill {buf[2]/waves:7.0f}  tiles/wave "
              f"{tiles/waves:5.2f}  wave life {buf[3]/waves:9.0f} cyc", flush=True)


if __name__ == "__main__":
    main()
