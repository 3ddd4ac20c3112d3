"""Kernel inventory of UltraNet's module-level forward (UltraNetQua.forward_modules: Conv2d_Q on qvit_conv_wonly,
activation_quantize_fn on the HIP quantizer, BatchNorm2d / MaxPool2d on ATen kernels) and of Linear_Q, for
`rocprofv3 --kernel-trace --stats -- python tools/profile_ultra_modules.py`: the stats list every kernel the path
launches (no MIOpen / library convolution expected). Prints per-forward wall time too."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from quantized_vit_amd.quant_ultra import linear_Q_fn  # noqa: E402
from quantized_vit_amd.ultranet import random_ultranet, synthetic_images_u8  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    batch = int(os.environ.get("BATCH", "16"))
    model = random_ultranet(seed=0, device=dev, calib_batch=2, img_size=416)
    img = synthetic_images_u8(batch, 416, seed=1, device=dev)
    lin = linear_Q_fn(4)(1024, 1000).to(dev)
    x = torch.randn(batch * 197, 1024, device=dev)
    with torch.no_grad():
        for _ in range(2):
            model.forward_modules(img)
            lin(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        iters = 5
        for _ in range(iters):
            io, _ = model.forward_modules(img)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / iters
        t0 = time.perf_counter()
        for _ in range(iters):
            lin(x)
        torch.cuda.synchronize()
        dl = (time.perf_counter() - t0) / iters
    print(f"UltraNetQua.forward_modules b{batch} @416: {dt * 1e3:.2f} ms ({batch / dt:.1f} img/s); "
          f"Linear_Q [{x.shape[0]}x1024] -> 1000: {dl * 1e3:.3f} ms; io {tuple(io.shape)}")


if __name__ == "__main__":
    main()
