"""The split part of the one-product prefilter's bound (csrc/assign_mfma_impl.h x1_eps) on the
host: for fp32 and fp64 rows, |(||c||^2 + xh . th) - (||c||^2 + x . t)| (t = -2c, exact fp64
sums of exact products) stays below hx * ||t - th|| + ||x - xh|| * (||th|| + ||t - th||) with
the kernel's inputs: ||xh||, the row's own ||xl|| (or 2^-8 ||xh|| without it) and the largest
centroid hi / lo norms.  The hardware part (MFMA accumulation, tag bits) is priced from the
probe (tools/probe_mfma_acc.hip) and exercised by tests/test_x3_gpu.py."""
import math

import pytest
import torch

R8 = 2 ** -8 / (1 - 2 ** -8)


def _bf(t):
    return t.float().to(torch.bfloat16).double()


def _split_part(hx, lx, Hc, Lc):
    Tc = Lc * (1 + R8)
    dx = torch.where(lx >= 0, lx * (1 + R8), hx * (2 ** -8 + 2 ** -16))
    return hx * Tc + dx * (Hc + Tc)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("offset", [0.0, 50.0])
@pytest.mark.parametrize("own_xl", [True, False])
def test_one_product_split_bound(dtype, offset, own_xl):
    g = torch.Generator().manual_seed(3)
    n, d, k = 512, 128, 64
    x = (torch.randn(n, d, generator=g, dtype=torch.float64) * 3 + offset).to(dtype)
    c = (torch.randn(k, d, generator=g, dtype=torch.float64) * 3 + offset).to(dtype)
    x64, t64 = x.double(), -2 * c.double()
    xh = _bf(x64)
    xl = _bf((x64 - xh).to(dtype).double())  # the split kernel's lo term
    th = _bf(t64)
    tl = _bf((t64 - th).to(dtype).double())
    exact = x64 @ t64.T
    one = xh @ th.T
    err = (one - exact).abs()
    hx = xh.norm(dim=1) * 1.0001
    lx = xl.norm(dim=1) * 1.0001 if own_xl else torch.full((n,), -1.0, dtype=torch.float64)
    Hc = th.norm(dim=1).max() * 1.0001
    Lc = tl.norm(dim=1).max() * 1.0001
    bound = _split_part(hx, lx, Hc, Lc)
    assert torch.all(err <= bound[:, None]), float((err / bound[:, None]).max())
    # not vacuous: the observed split error uses a visible part of the bound
    assert float((err / bound[:, None]).max()) > 0.02
    if own_xl:  # the row's own residual is tighter than the worst case
        assert float(bound.mean()) < float(_split_part(hx, torch.full_like(lx, -1.0), Hc, Lc).mean())
