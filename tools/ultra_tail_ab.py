"""UltraNet @416 b256: the fused forward with layers.16-28 in one launch (qvit_ultra_tail) against the same
library's per-layer launches (ultranet.TAIL_MAX = 0), alternating, HIP events (median of 10 per arm and round)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import quantized_vit_amd.ultranet as un  # noqa: E402


def median_ms(fn, iters=10):
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
    dev = torch.device("cuda:0")
    model = un.random_ultranet(seed=0, device=dev)
    x = un.synthetic_images_u8(256, 416, seed=1, device=dev)
    saved = un.TAIL_MAX
    with torch.no_grad():
        for r in range(3):
            for tail in (True, False):
                un.TAIL_MAX = saved if tail else 0
                ms = median_ms(lambda: model.forward_fused(x))
                print(f"round {r} {'tail' if tail else 'per-layer'}: {ms:.3f} ms/forward  {256 / ms * 1e3:.0f} img/s",
                      flush=True)
    un.TAIL_MAX = saved


if __name__ == "__main__":
    main()
