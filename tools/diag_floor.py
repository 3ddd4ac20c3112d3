"""Diagnostic: the oracle's fp32-vs-fp64 'floor' on the bench's parity images, per layer.

Runs the oracle (oracle/quant_oracle.py) in fp32 and in fp64 on the seed-12345 b2 images with every activation
quantizer's codes captured, and prints the code flips per layer and the logits' distance. `--device cuda` builds
(calibrates) the model on the GPU exactly as bench.py does; the oracle itself always runs on the CPU.
Also compares the quantizer scalars of the device-built and CPU-built models.

    python tools/diag_floor.py vit_large_patch16_384 --device cuda
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import quant_oracle as O  # noqa: E402
from quantized_vit_amd.calibrate import VIT_CONFIGS, build_quantized_vit, synthetic_images  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("model")
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--no-hook", action="store_true")
    a = ap.parse_args()
    mc = VIT_CONFIGS[a.model]
    cfg = O.ViTConfig(img_size=mc["img_size"], patch_size=mc["patch_size"], embed_dim=mc["embed_dim"],
                      depth=mc["depth"], num_heads=mc["num_heads"])
    dev = torch.device(a.device)
    model = build_quantized_vit(a.model, seed=0, device=dev)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    if dev.type != "cpu":
        sdc = {k: v.detach() for k, v in build_quantized_vit(a.model, seed=0).state_dict().items()}
        diffs = [(k, float(sd[k].reshape(-1)[0]), float(sdc[k].reshape(-1)[0])) for k in sd
                 if ("quant" in k or "q_m" in k) and not torch.equal(sd[k], sdc[k])]
        print(f"quantizer scalars differing between device- and CPU-built models: {len(diffs)}")
        for k, x, y in diffs[:12]:
            print(f"  {k}: device {x!r} cpu {y!r}")
    img = synthetic_images(2, mc["img_size"], seed=12345)
    codes = {}

    def hook_for(tag):
        def hook(prefix, x, q):
            if q.quant_mode != O.WEIGHT_AND_ACTIVATION:
                return x
            k = O.quant_codes(x, q.quant_type, q.d_act, q.q_m_act, q.t_act)
            codes[(tag, prefix)] = k
            return O._t(q.d_act).to(x.dtype) * k
        return hook
    with torch.no_grad():
        if a.no_hook:
            r32 = O.vit_forward(sd, cfg, img)
            r64 = O.vit_forward({k: v.double() for k, v in sd.items()}, cfg, img.double())
        else:
            r32 = O.vit_forward(sd, cfg, img, act_hook=hook_for(32))
            r64 = O.vit_forward({k: v.double() for k, v in sd.items()}, cfg, img.double(), act_hook=hook_for(64))
    print(f"logits rel fp32 vs fp64: {((r32.double() - r64).norm() / r64.norm()).item():.3e}; "
          f"|logits| max {r64.abs().max().item():.3e} std {r64.std().item():.3e}")
    tot = 0
    for (tag, p), k in codes.items():
        if tag != 32:
            continue
        k64 = codes[(64, p)]
        n = int((k != k64).sum())
        tot += n
        print(f"{p}: flips {n} of {k.numel()}, nonzero codes {(k != 0).float().mean().item():.3f}, "
              f"saturated {(k.abs() >= k.abs().max()).float().mean().item():.3f}, max|code| {int(k.abs().max())}")
    print("total flips", tot)


if __name__ == "__main__":
    main()
