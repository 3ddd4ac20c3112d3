"""The tie classifier the GPU parity tests rely on (tests/parity_tools.py), on the CPU."""
import torch

from oracle import quant_oracle as O
from parity_tools import TIE_TOL, tie_check


def test_tie_check_accepts_only_one_step_flips_at_boundaries():
    d, qm = 0.01, 1.0
    x = torch.tensor([0.0150000004, 0.0251, 0.3333, -0.4449999, 0.7, 0.00499999])
    own = O.quant_codes(x, O.LINEAR, d, qm)
    got = own.clone()
    st = tie_check(x, got, own, O.LINEAR, d, qm, 1.0)
    assert st == {"flips": 0, "non_ties": 0, "max_dist": 0.0, "total": 6, "cr_explained": 0}
    got[0] = own[0] + 1 if own[0] == 1 else own[0] - 1      # 1.5 code units: a tie
    got[3] = -45 if own[3] == -44 else -44                   # -44.49999: a tie
    got[5] = 1 - own[5] if own[5] == 0 else 0               # 0.499999 code units: a tie (0 <-> 1)
    st = tie_check(x, got, own, O.LINEAR, d, qm, 1.0)
    assert st["flips"] == 3 and st["non_ties"] == 0 and st["max_dist"] <= TIE_TOL
    got[2] = own[2] + 1                                       # 33.33: far from a boundary
    assert tie_check(x, got, own, O.LINEAR, d, qm, 1.0)["non_ties"] == 1
    got[2] = own[2]
    got[4] = own[4] + 2                                       # two steps
    assert tie_check(x, got, own, O.LINEAR, d, qm, 1.0)["non_ties"] == 1


def test_tie_check_nonlinear_domain():
    d, qm, t = 0.02, 1.5, 0.9
    k = 17
    x = torch.tensor([((k + 0.5) * d) ** (1 / t)], dtype=torch.float32)   # at the boundary in |x|^t
    own = O.quant_codes(x, O.NONLINEAR, d, qm, t)
    other = torch.tensor([float(2 * k + 1) - own.item()])
    assert tie_check(x, other, own, O.NONLINEAR, d, qm, t)["non_ties"] == 0
    x2 = torch.tensor([((k + 0.3) * d) ** (1 / t)])
    own2 = O.quant_codes(x2, O.NONLINEAR, d, qm, t)
    assert tie_check(x2, own2 + 1, own2, O.NONLINEAR, d, qm, t)["non_ties"] == 1


def test_cr_codes_is_the_correctly_rounded_quantizer():
    """cr_codes (the flip classifier) = the quantizer with log/exp rounded once from fp64, which agrees with the
    oracle's torch codes except where torch's exp(log(a)) is not the correctly rounded composition."""
    from oracle.ties import cr_codes
    g = torch.Generator().manual_seed(4)
    x = torch.randn(200_000, generator=g)
    d, qm, t = 3.0 / 127, 3.0, 1.0
    own = O.quant_codes(x, O.NONLINEAR, d, qm, t)
    cr = cr_codes(x, O.NONLINEAR, d, qm, t)
    diff = cr != own
    assert int(diff.sum()) <= 1e-4 * x.numel()
    if bool(diff.any()):   # only at ties, one step
        pos = (x[diff].double().abs() / d)
        assert float((pos - (torch.minimum(cr[diff].abs(), own[diff].abs()).double() + 0.5)).abs().max()) < 1e-4
        assert float((cr[diff] - own[diff]).abs().max()) == 1
    # saturation / zero masks as the reference's
    edge = torch.tensor([0.0, -0.0, 3.0, -3.5, 100.0])
    assert torch.equal(cr_codes(edge, O.NONLINEAR, d, qm, t), O.quant_codes(edge, O.NONLINEAR, d, qm, t))
    assert torch.equal(cr_codes(x, O.LINEAR, d, qm, t), O.quant_codes(x, O.LINEAR, d, qm, t))
