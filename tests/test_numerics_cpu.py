"""CPU numerics against the reference math (fp64 oracles restating `src/common.py` / `src/model.py`)."""
import math

import pytest
import torch

from masters_thesis_amd.data.common import (add_quadratic_features, gaussian_nll_dense, inverse_returns_covariance,
                                            lookback_target_split, ols, ols_features, woodbury_nll_closed_form)
from masters_thesis_amd.ops.losses import decoder_losses


def _pinv_ols(X, y):
    """The reference's exact estimator (`src/common.py:33-47`)."""
    X = X.unsqueeze(0) if X.dim() == 1 else X
    y = y.unsqueeze(0) if y.dim() == 2 else y
    Xd = torch.stack([torch.ones_like(X), X], dim=-1)
    sol = torch.linalg.pinv(Xd.mT @ Xd) @ (Xd.mT @ y.mT)
    return sol[:, 0, :], sol[:, 1, :]


def test_closed_form_ols_equals_pinv():
    torch.manual_seed(0)
    X = torch.randn(7, 30, dtype=torch.float64)
    y = torch.randn(7, 11, 30, dtype=torch.float64) + 0.5 * X.unsqueeze(1)
    a, b = ols(X, y)
    ra, rb = _pinv_ols(X, y)
    torch.testing.assert_close(a, ra)
    torch.testing.assert_close(b, rb)
    # unbatched squeeze semantics + degenerate (constant) regressor follows pinv's min-norm solution
    Xc = torch.full((30,), 0.7, dtype=torch.float64)
    yc = torch.randn(5, 30, dtype=torch.float64)
    a1, b1 = ols(Xc, yc)
    ra1, rb1 = _pinv_ols(Xc, yc)
    torch.testing.assert_close(a1, ra1.squeeze())
    torch.testing.assert_close(b1, rb1.squeeze())


def test_woodbury_closed_form_matches_dense_logdet():
    torch.manual_seed(1)
    K, n = 100, 30
    alpha = torch.randn(K, dtype=torch.float64) * 0.1
    beta = torch.randn(K, dtype=torch.float64) * 0.3 + 1
    w = torch.rand(K, dtype=torch.float64) * 5 + 0.5
    fm, fv = torch.tensor(0.05, dtype=torch.float64), torch.tensor(0.3, dtype=torch.float64)
    r = torch.randn(K, n, dtype=torch.float64)
    a1, b1 = alpha.clone().requires_grad_(), beta.clone().requires_grad_()
    dense = gaussian_nll_dense((a1 + b1 * fm).unsqueeze(-1),
                               inverse_returns_covariance(b1.unsqueeze(-1), torch.diag(w), fv), r)
    ga, gb = torch.autograd.grad(dense, (a1, b1))
    a2, b2 = alpha.clone().requires_grad_(), beta.clone().requires_grad_()
    closed = woodbury_nll_closed_form(a2, b2, fm, fv, w, r)
    ga2, gb2 = torch.autograd.grad(closed, (a2, b2))
    assert abs(closed.item() - dense.item()) < 1e-9 * abs(dense.item())
    torch.testing.assert_close(ga2, ga, rtol=1e-9, atol=1e-10)
    torch.testing.assert_close(gb2, gb, rtol=1e-9, atol=1e-10)


@pytest.mark.parametrize("B,mode", [(1, "reference"), (2, "reference"), (2, "per_window")])
def test_decoder_losses_cpu_path(B, mode):
    torch.manual_seed(2)
    K, n = 20, 30
    N = B * K
    ab = torch.randn(N, 2, dtype=torch.float64)
    y = torch.randn(N, n, 4, dtype=torch.float64)
    factor = torch.stack([torch.randn(B) * 0.1, torch.rand(B) + 0.2], -1).double()
    inv_psi = torch.rand(N, dtype=torch.float64) + 1
    mse, nll, mae = decoder_losses(ab, y, factor, inv_psi, batch_windows=B, nll_mode=mode)
    pred = ab[:, :1] + ab[:, 1:] * y[..., 1]
    assert abs(mse.item() - ((pred - y[..., 0]) ** 2).mean().item()) < 1e-12
    assert abs(mae.item() - (pred - y[..., 0]).abs().mean().item()) < 1e-12
    if mode == "reference":
        fac = factor.flatten()
        ref = gaussian_nll_dense(ab[:, :1] + ab[:, 1:] * fac[0],
                                 inverse_returns_covariance(ab[:, 1:], torch.diag(inv_psi), fac[1]), y[..., 0])
    else:
        ref = sum(gaussian_nll_dense(ab[w * K:(w + 1) * K, :1] + ab[w * K:(w + 1) * K, 1:] * factor[w, 0],
                                     inverse_returns_covariance(ab[w * K:(w + 1) * K, 1:],
                                                                torch.diag(inv_psi[w * K:(w + 1) * K]), factor[w, 1]),
                                     y[w * K:(w + 1) * K, :, 0]) for w in range(B))
    assert abs(nll.item() - ref.item()) < 1e-8 * abs(ref.item())


def test_windowing_shapes_and_features():
    K, Nd = 4, 1000
    rs = torch.randn(K, Nd)
    rm = torch.randn(Nd)
    X, y = lookback_target_split(rs, rm, 60, 30, 90, True)
    assert X.shape == (Nd // 90, K, 60, 2) and y.shape == (Nd // 90, K, 30, 2)
    assert torch.equal(X[1, 2, 0, 0], rs[2, 90])
    assert torch.equal(y[1, 2, 0, 1], rm[150])
    Xq = add_quadratic_features(X, interaction_only=True)
    assert Xq.shape[-1] == 3 and torch.allclose(Xq[..., 2], X[..., 0] * X[..., 1])
    assert add_quadratic_features(X, interaction_only=False).shape[-1] == 5
    Xr, yr = lookback_target_split(rs, rm, 60, 30, 10, False)
    assert Xr.shape[2] == 60 and yr.shape[2] == 30 and torch.equal(yr[0, 0, 0, 0], rs[0, 30])
    a, b, factor, inv_psi = ols_features(y)
    assert a.shape == (Nd // 90, K) and factor.shape == (Nd // 90, 2) and inv_psi.shape == (Nd // 90, K)
    torch.testing.assert_close(factor[:, 1], y[:, 0, :, 1].var(dim=-1))


def test_fused_adam_cpu_matches_torch():
    from masters_thesis_amd.ops.optim import FlatParameters, FusedAdam

    torch.manual_seed(3)
    shapes = [(16, 3), (16,), (1, 4)]
    ref = [torch.nn.Parameter(torch.randn(s)) for s in shapes]
    mine = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    o_ref = torch.optim.Adam(ref, lr=1e-2, weight_decay=1e-3)
    flat = FlatParameters(mine)
    o = FusedAdam(flat, lr=1e-2, weight_decay=1e-3)
    for step in range(4):
        gs = [torch.randn(s) * (5 if step % 2 else 0.2) for s in shapes]
        for p, g in zip(ref, gs):
            p.grad = g.clone()
        torch.nn.utils.clip_grad_norm_(ref, 1.0)
        o_ref.step()
        flat.zero_grad()
        for p, g in zip(mine, gs):
            p.grad.copy_(g)
        o.step(max_norm=1.0)
    for a, b in zip(mine, ref):
        torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-5, atol=1e-6)
    sd = o.state_dict()
    assert set(sd["state"][0]) == {"step", "exp_avg", "exp_avg_sq"} and sd["param_groups"][0]["lr"] == 1e-2


def test_plateau_matches_torch_scheduler():
    from masters_thesis_amd.engine.schedulers import PlateauScheduler
    from masters_thesis_amd.ops.optim import FlatParameters, FusedAdam

    p = torch.nn.Parameter(torch.zeros(4))
    o_ref = torch.optim.Adam([p], lr=1.0)
    s_ref = torch.optim.lr_scheduler.ReduceLROnPlateau(o_ref, mode="min", factor=0.5, patience=2)
    q = torch.nn.Parameter(torch.zeros(4))
    o = FusedAdam(FlatParameters([q]), lr=1.0)
    s = PlateauScheduler.from_torch(s_ref, o)
    for v in [5, 4, 4.5, 4.4, 4.3, 4.2, 4.6, 4.7, 4.8, 3.0, 3.1, 3.2, 3.3, 3.4]:
        s_ref.step(v)
        s.step(v)
        assert math.isclose(o.lr, o_ref.param_groups[0]["lr"])
    assert o.lr < 1.0
