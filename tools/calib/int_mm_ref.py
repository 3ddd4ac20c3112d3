"""Calibration: the vendor library's int8 x int8 -> int32 GEMM (torch._int_mm -> hipBLASLt) on the ViT-B/16 b256
GEMM shapes, timed with HIP events on the current stream (median of 20). A reference point for what the
library reaches on the same matrix cores with no int4 unpack and no fused epilogue. Diagnostic only."""
import torch

PEAK = 256 * 4 * 2048 * 2.4e9 / 1e12


def main():
    dev = torch.device("cuda:0")
    for name, (M, N, K) in {"fc1": (50432, 3072, 768), "fc2": (50432, 768, 3072), "qkv": (50432, 2304, 768),
                            "vitl_fc1": (73856, 4096, 1024)}.items():
        A = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
        for layout in ("nt", "nn"):
            if layout == "nt":
                B = torch.randint(-7, 8, (N, K), dtype=torch.int8, device=dev).t()   # [K, N] column-major
            else:
                B = torch.randint(-7, 8, (K, N), dtype=torch.int8, device=dev)
            try:
                C = torch._int_mm(A, B)
            except Exception as e:  # noqa: BLE001
                print(f"{name} {layout}: _int_mm refused: {e}")
                continue
            ts = []
            for _ in range(23):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                torch._int_mm(A, B, out=C) if hasattr(torch, "_int_mm") else None
                e.record()
                e.synchronize()
                ts.append(s.elapsed_time(e) * 1e3)
            t = sorted(ts[3:])[len(ts[3:]) // 2]
            tops = 2 * M * N * K / t / 1e6
            print(f"{name:9s} {layout} M={M} N={N} K={K}: {t:8.1f} us  {tops:7.1f} TOPS  {tops / PEAK * 100:5.1f} % of int8 peak",
                  flush=True)


if __name__ == "__main__":
    main()
