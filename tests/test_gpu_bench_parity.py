"""Parity on the bench's own images: bench.py's parity_report on the seed-12345 b2 images of the
headline workload (ViT-B/16 @224, configs[1]) and of configs[3] (ViT-L/16 @384), with the model built exactly as
bench.py builds it (calibrated on the device). The bench line's `parity.tie_resolved.pass` is this test's
criterion: every differing activation code a proven rounding tie, no layer over the 1e-4 flip budget
(oracle/ties.py), logits within the north star's 1e-3 once ties resolve alike (here: 2e-5).

Reference: QViT_with_GETA/vit_model.py:125-175 (the blocks), OTO/quantization/quant_layers.py:41-69,356-381.
"""
import pytest

import bench
from quantized_vit_amd.calibrate import build_quantized_vit

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,img_size", [("vit_base_patch16_224", 224), ("vit_large_patch16_384", 384)])
def test_bench_parity_images(dev, name, img_size):
    model = build_quantized_vit(name, seed=0, device=dev)
    rep = bench.parity_report(model, name, img_size, dev)
    u, t = rep["untied"], rep["tie_resolved"]
    print(f"{name}: untied rel {u['rel_device_weights']:.3e} (oracle weights {u['rel_oracle_weights']:.3e}, "
          f"floor {u['floor_fp32_vs_fp64']:.3e}); weight flips {u['weight_code_flips']['flips']} "
          f"({u['weight_code_flips']['cr_explained']} explained by correctly rounded exp/log); tie-resolved rel "
          f"{t['rel']:.3e}, {t['tie_flips']} tie flips ({t['cr_explained']} by exp/log) of {t['codes']}; "
          f"over budget {t['layers_over_budget']}")
    assert not t["missing_layers"]
    assert t["non_tie_differences"] == 0
    assert not t["layers_over_budget"], t["layers_over_budget"]
    assert t["rel"] <= 2e-5
    assert t["pass"]
