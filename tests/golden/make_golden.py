"""Generates the golden regression fixtures in tests/golden/ from the CPU oracle.

    python tests/golden/make_golden.py

quantizer_vectors.npz: inputs, parameters and expected integer codes of the reference quantizers
  (SymQuantizerLinear / SymQuantizerNonLinear restated in oracle/quant_oracle.py), including
  exact rounding-boundary inputs (x/d = n + 0.5), zeros, saturation and negative q_m.
vit_tiny_b2_logits.npz: seeds/config and the oracle's logits of a 2-block ViT-Tiny/16 W4A8
  (nonlinear quantizer) built by quantized_vit_amd.calibrate.build_quantized_vit on the CPU.
These are regression vectors of the restatement, not outputs of the reference (import denied).
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import quant_oracle as O  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def quantizer_vectors():
    g = torch.Generator().manual_seed(1234)
    cases = []
    for qt, d, qm, t in [(O.LINEAR, 0.05, 1.0, 1.0), (O.LINEAR, 1 / 127, 1.0, 1.0), (O.NONLINEAR, 0.05, 1.0, 1.0),
                         (O.NONLINEAR, 0.021, 0.9, 0.8), (O.NONLINEAR, 0.11, 2.5, 1.2), (O.LINEAR, 0.2, -1.0, 1.0)]:
        x = torch.randn(4096, generator=g) * qm * 0.6
        # rounding boundaries: x = (n + 0.5) * d exactly representable cases and near them
        n = torch.arange(-20, 20, dtype=torch.float32)
        x = torch.cat([x, (n + 0.5) * d, torch.tensor([0.0, -0.0, qm, -qm, 10 * abs(qm), -10 * abs(qm)])])
        codes = O.quant_codes(x, qt, d, qm, t)
        cases.append((qt, (d, qm, t), x.numpy(), codes.numpy().astype(np.int32)))
    arrs = {"n_cases": np.array(len(cases))}
    for i, (qt, p, x, c) in enumerate(cases):
        arrs[f"qtype_{i}"] = np.array(qt)
        arrs[f"params_{i}"] = np.array(p, dtype=np.float64)
        arrs[f"x_{i}"] = x
        arrs[f"codes_{i}"] = c
    np.savez_compressed(os.path.join(OUT, "quantizer_vectors.npz"), **arrs)


def vit_tiny():
    from quantized_vit_amd.calibrate import build_quantized_vit, synthetic_images
    seed, depth, ncls, batch, img_seed = 0, 2, 1000, 2, 7
    model = build_quantized_vit("vit_tiny_patch16_224", num_classes=ncls, seed=seed, depth=depth)
    sd = {k: v.detach() for k, v in model.state_dict().items()}
    cfg = O.ViTConfig(embed_dim=192, depth=depth, num_heads=3, num_classes=ncls)
    img = synthetic_images(batch, 224, seed=img_seed)
    with torch.no_grad():
        logits = O.vit_forward(sd, cfg, img)
    np.savez_compressed(os.path.join(OUT, "vit_tiny_b2_logits.npz"), seed=seed, depth=depth, num_classes=ncls,
                        batch=batch, img_seed=img_seed, logits=logits.numpy())


if __name__ == "__main__":
    quantizer_vectors()
    vit_tiny()
    print("written to", OUT)
