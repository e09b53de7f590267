"""Dataset-build kernels (csrc/data.hip): OLS features vs the PyTorch formulation, DGP distribution moments."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _native():
    from masters_thesis_amd.ops import _lib

    assert _lib.lib(required=True) is not None


def test_ols_features_matches_torch():
    from masters_thesis_amd.data.common import ols_features as ref
    from masters_thesis_amd.ops import ols

    g = torch.Generator().manual_seed(0)
    W, K, n, C = 37, 100, 60, 2
    mkt = torch.randn(W, 1, n, generator=g) * 0.5 + 0.07
    a = torch.randn(W, K, 1, generator=g) * 0.1
    b = torch.randn(W, K, 1, generator=g) * 0.35 + 0.9
    rs = a + b * mkt + 0.3 * torch.randn(W, K, n, generator=g)
    y = torch.stack([rs, mkt.expand(W, K, n)], dim=-1).contiguous()
    want = [t.double() for t in ref(y.double())]
    got = ols.ols_features(y.to(DEV))
    for gt, wt, name in zip(got, want, ("alphas", "betas", "factor", "inv_psi")):
        torch.testing.assert_close(gt.double().cpu(), wt, rtol=2e-4, atol=2e-5, msg=name)


def test_ols_features_constant_market_pinv_branch():
    from masters_thesis_amd.data.common import ols_features as ref
    from masters_thesis_amd.ops import ols

    W, K, n = 2, 8, 10
    rs = torch.randn(W, K, n, dtype=torch.float64)
    mkt = torch.full((W, K, n), 0.5, dtype=torch.float64)
    y = torch.stack([rs, mkt], dim=-1)
    want = ref(y)
    got = ols.ols_features(y.float().to(DEV))
    torch.testing.assert_close(got[0].double().cpu(), want[0], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(got[1].double().cpu(), want[1], rtol=1e-4, atol=1e-5)


def test_dgp_moments_and_determinism():
    from masters_thesis_amd.data.dgp import SyntheticLogReturns as S

    K, N = 64, 200_000
    r_s, r_m, al, be = S.generate(K, N, device=DEV, seed=7)
    r_s2, r_m2, _, _ = S.generate(K, N, device=DEV, seed=7)
    assert torch.equal(r_s, r_s2) and torch.equal(r_m, r_m2)
    r_s3, _, _, _ = S.generate(K, N, device=DEV, seed=8)
    assert not torch.equal(r_s, r_s3)
    assert torch.isfinite(r_s).all() and torch.isfinite(r_m).all()
    mk, idio = S.mkt_params, S.idio_params
    df = mk["df"]
    t_var = df / (df - 2)
    m = r_m.double()
    assert abs(m.mean().item() - mk["loc"]) < 5 * mk["scale"] * math.sqrt(t_var / N)
    assert abs(m.var().item() / (mk["scale"] ** 2 * t_var) - 1) < 0.05
    # residuals given the true coefficients are the idiosyncratic t-variates
    eps = (r_s.double() - al.double()[:, None] - be.double()[:, None] * m[None, :])
    assert abs(eps.mean().item() - idio["loc"]) < 5 * idio["scale"] * math.sqrt(t_var / (K * N))
    assert abs(eps.var().item() / (idio["scale"] ** 2 * t_var) - 1) < 0.03
    # Student-t(5) excess kurtosis is 6: a normal sampler would give ~0
    z = (eps - eps.mean()) / eps.std()
    assert (z ** 4).mean().item() - 3 > 3.0
    # independence of market and idiosyncratic noise
    assert abs(torch.corrcoef(torch.stack([eps[0], m]))[0, 1].item()) < 0.02
    big_K = 4096
    _, _, al_b, be_b = S.generate(big_K, 16, device=DEV, seed=3)
    ap, bp = S.alpha_params, S.beta_params
    assert abs(al_b.double().mean().item() - ap["loc"]) < 5 * ap["scale"] / math.sqrt(big_K)
    assert abs(be_b.double().std().item() / bp["scale"] - 1) < 0.06
