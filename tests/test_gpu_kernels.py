"""Numerics of the HIP kernels against plain PyTorch fp64 references (run on the MI355X box).

Every test asserts that the native extension is the code path that ran (no silent
eager fallback): ``masters_thesis_amd._C`` must be importable and the ops must be
dispatched to it for CUDA tensors.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _native():
    from masters_thesis_amd.ops import _lib

    assert _lib.lib(required=True) is not None
    assert not _lib.fallback_allowed()


def _lstm_weights(F, H, L, seed=0):
    g = torch.Generator().manual_seed(seed)
    k = 1.0 / math.sqrt(H)
    ws = []
    for l in range(L):
        fin = F if l == 0 else H
        for shape in ((4 * H, fin), (4 * H, H), (4 * H,), (4 * H,)):
            ws.append((torch.rand(shape, generator=g) * 2 - 1) * k)
    return ws


def _ref_lstm(x, ws, L):
    """fp64 CPU reference via the nn.LSTM kernel."""
    x64 = x.detach().double().cpu().requires_grad_(True)
    w64 = [w.detach().double().cpu().requires_grad_(True) for w in ws]
    N, H = x.shape[0], ws[1].shape[1]
    h0 = torch.zeros(L, N, H, dtype=torch.float64)
    out, _, _ = torch._VF.lstm(x64, (h0, h0), w64, True, L, 0.0, False, False, True)
    return out[:, -1], x64, w64


# "high" = PyTorch's TF32-class setting: the pipelined forward runs fp16 activations x fp16 hi+lo weights (PREC_F16X2);
# "bf16x3" = the ~fp32-accurate 3-pass form
TOLS = {"highest": 2e-5, "high": 1e-3, "bf16x3": 3e-4, "medium": 3e-2}


@pytest.mark.parametrize("prec", ["highest", "high", "bf16x3", "medium"])
@pytest.mark.parametrize("N,T,F,H,L", [(100, 60, 3, 64, 2), (37, 20, 5, 64, 1), (40, 15, 3, 32, 3),
                                       (33, 12, 64, 128, 2), (300, 60, 3, 64, 4)])
def test_lstm_forward_backward(prec, N, T, F, H, L):
    from masters_thesis_amd.ops.lstm import lstm_last_hidden

    torch.manual_seed(1)
    x = torch.randn(N, T, F)
    ws = _lstm_weights(F, H, L)
    R = torch.randn(N, H)
    ref, x64, w64 = _ref_lstm(x, ws, L)
    (ref * R.double()).sum().backward()

    xg = x.to(DEV).requires_grad_(True)
    wg = [w.to(DEV).requires_grad_(True) for w in ws]
    out = lstm_last_hidden(xg, wg, L, 0.0, True, prec)
    (out * R.to(DEV)).sum().backward()
    tol = TOLS[prec]
    scale = ref.abs().max().item()
    err = (out.double().cpu() - ref.detach()).abs().max().item()
    assert err <= tol * max(scale, 1.0), f"forward err {err} (scale {scale})"
    for name, a, b in [("x", xg.grad, x64.grad)] + [(f"w{i}", wg[i].grad, w64[i].grad) for i in range(len(ws))]:
        sc = b.abs().max().item()
        e = (a.double().cpu() - b).abs().max().item()
        assert e <= 4 * tol * max(sc, 1e-3) + 1e-6, f"grad {name}: err {e} (scale {sc})"


def test_lstm_dropout_path():
    from masters_thesis_amd.ops.lstm import lstm_last_hidden

    torch.manual_seed(2)
    x = torch.randn(64, 30, 3, device=DEV, requires_grad=True)
    ws = [w.to(DEV).requires_grad_(True) for w in _lstm_weights(3, 64, 3)]
    out_eval = lstm_last_hidden(x, ws, 3, 0.3, False, "highest")
    out_nodrop = lstm_last_hidden(x, ws, 3, 0.0, True, "highest")
    torch.testing.assert_close(out_eval, out_nodrop, rtol=0, atol=0)
    out = lstm_last_hidden(x, ws, 3, 0.3, True, "highest")
    assert not torch.allclose(out, out_eval)
    out.sum().backward()
    assert all(torch.isfinite(w.grad).all() for w in ws)


@pytest.mark.parametrize("B,mode", [(1, "reference"), (3, "reference"), (3, "per_window"), (12, "reference"),
                                    (12, "per_window")])
def test_decoder_losses_match_dense_reference(B, mode):
    from masters_thesis_amd.data.common import gaussian_nll_dense, inverse_returns_covariance
    from masters_thesis_amd.ops.losses import decoder_losses

    torch.manual_seed(3)
    K, n = 100, 30
    N = B * K
    ab = torch.randn(N, 2, dtype=torch.float64) * 0.3 + torch.tensor([0.0, 1.0], dtype=torch.float64)
    y = torch.randn(N, n, 4, dtype=torch.float64)
    factor = torch.stack([torch.randn(B) * 0.1, torch.rand(B) * 0.5 + 0.2], -1).double()
    inv_psi = (torch.rand(N) * 5 + 1).double()

    # fp64 dense reference (exactly the reference's math, src/model.py:45-69)
    ab_r = ab.clone().requires_grad_(True)
    r, rm = y[..., 0], y[..., 1]
    pred = ab_r[:, :1] + ab_r[:, 1:] * rm
    mse_r = ((pred - r) ** 2).mean()
    if mode == "reference":
        fm, fv = factor.flatten()[0], factor.flatten()[1]
        nll_r = gaussian_nll_dense(ab_r[:, :1] + ab_r[:, 1:] * fm,
                                   inverse_returns_covariance(ab_r[:, 1:], torch.diag(inv_psi), fv), r)
    else:
        nll_r = 0
        for w in range(B):
            sl = slice(w * K, (w + 1) * K)
            fm, fv = factor[w, 0], factor[w, 1]
            nll_r = nll_r + gaussian_nll_dense(ab_r[sl, :1] + ab_r[sl, 1:] * fm,
                                               inverse_returns_covariance(ab_r[sl, 1:], torch.diag(inv_psi[sl]), fv),
                                               r[sl])
    (g_ref,) = torch.autograd.grad(mse_r * 0.7 + nll_r * 1.3, ab_r)

    abg = ab.float().to(DEV).requires_grad_(True)
    mse, nll, mae = decoder_losses(abg, y.float().to(DEV), factor.float().to(DEV), inv_psi.float().to(DEV),
                                   batch_windows=B, nll_mode=mode)
    (mse * 0.7 + nll * 1.3).backward()
    assert abs(mse.item() - mse_r.item()) <= 1e-5 * abs(mse_r.item())
    assert abs(nll.item() - nll_r.item()) <= 2e-5 * abs(nll_r.item()) + 1e-3
    assert abs(mae.item() - (pred - r).abs().mean().item()) <= 1e-5
    err = (abg.grad.double().cpu() - g_ref).abs().max().item()
    assert err <= 2e-4 * g_ref.abs().max().item(), err


def test_fused_adam_matches_torch_adam_with_clipping():
    from masters_thesis_amd.ops.optim import FlatParameters, FusedAdam

    torch.manual_seed(4)
    shapes = [(256, 3), (256, 64), (256,), (1, 64), (1,)]
    ref = [torch.nn.Parameter(torch.randn(s, device=DEV)) for s in shapes]
    mine = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    opt_ref = torch.optim.Adam(ref, lr=3e-3, weight_decay=1e-2)
    flat = FlatParameters(mine)
    opt = FusedAdam(flat, lr=3e-3, weight_decay=1e-2)
    for step in range(5):
        grads = [torch.randn(s, device=DEV) * (10 if step % 2 else 0.1) for s in shapes]
        for p, g in zip(ref, grads):
            p.grad = g.clone()
        torch.nn.utils.clip_grad_norm_(ref, 1.0)
        opt_ref.step()
        flat.zero_grad()
        for p, g in zip(mine, grads):
            p.grad.copy_(g)
        opt.step(max_norm=1.0)
    for a, b in zip(mine, ref):
        torch.testing.assert_close(a.detach(), b.detach(), rtol=2e-5, atol=2e-6)
    assert float(opt.step_t.item()) == 5.0


@pytest.mark.parametrize("n_params", [51_074, 3_000_000, 12_980_226])  # small LSTM, mid, mlp_large
def test_single_launch_adam_matches_two_launch_and_zeroes_grads(n_params, monkeypatch):
    """csrc/optim.hip adam_fused_kernel (in-launch norm ticket, grid <= 256 workgroups) against the two-launch
    norm + update pair, over several steps (the monotonic ticket spans launches), with grad zeroing."""
    from masters_thesis_amd.ops.optim import FlatParameters, FusedAdam

    torch.manual_seed(6)
    opts = []
    for single in (False, True):
        ps = [torch.nn.Parameter(torch.full((n_params,), 0.5, device=DEV))]
        flat = FlatParameters(ps)
        opts.append((flat, FusedAdam(flat, lr=1e-3, weight_decay=1e-5, single_launch=single)))
    assert not opts[0][1].single_launch and opts[1][1].single_launch
    for step in range(4):
        g = torch.randn(opts[0][0].padded, device=DEV) * (3.0 if step % 2 else 0.01)
        for flat, opt in opts:
            flat.grad.copy_(g)
            opt.step(max_norm=5.0, zero_grad=True)
    (fa, oa), (fb, ob) = opts
    torch.testing.assert_close(fb.data, fa.data, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(ob.grad_norm, oa.grad_norm, rtol=1e-5, atol=0)
    assert ob.grads_zeroed and float(fb.grad.abs().max()) == 0.0
    assert float(ob.step_t.item()) == 4.0 and int(ob.ticket.item()) > 0
    assert float(ob.sync_timeouts.item()) == 0.0 and float(ob.nonfinite.item()) == 0.0


def test_flat_grads_survive_backward():
    from masters_thesis_amd.ops.optim import FlatParameters

    lin = torch.nn.Linear(8, 4).to(DEV)
    flat = FlatParameters(lin.parameters())
    ptr = lin.weight.grad.data_ptr()
    lin(torch.randn(3, 8, device=DEV)).sum().backward()
    assert lin.weight.grad.data_ptr() == ptr
    assert flat.grad.abs().sum() > 0


@pytest.mark.parametrize("coeffs", [(0.0, 1.0), (1.0, 0.0), (1.0, 100.0)])
def test_heads_losses_grads_and_metric_accumulator(coeffs):
    from masters_thesis_amd.ops.losses import heads_losses

    torch.manual_seed(5)
    N, H, n = 100, 64, 30
    h = torch.randn(N, H, dtype=torch.float64) * 0.5
    wa, ba = torch.randn(1, H, dtype=torch.float64) * 0.1, torch.randn(1, dtype=torch.float64) * 0.1
    wb, bb = torch.randn(1, H, dtype=torch.float64) * 0.1, torch.ones(1, dtype=torch.float64)
    y = torch.randn(N, n, 4, dtype=torch.float64)
    factor = torch.tensor([[0.05, 0.3]], dtype=torch.float64)
    inv_psi = torch.rand(N, dtype=torch.float64) * 3 + 1
    ref_in = [t.clone().requires_grad_(True) for t in (h, wa, ba, wb, bb)]
    ab, mse_r, nll_r, _, tot_r = heads_losses(*ref_in, y, factor, inv_psi, c_nll=coeffs[0], c_mse=coeffs[1])
    tot_r.backward()
    gin = [t.float().to(DEV).requires_grad_(True) for t in (h, wa, ba, wb, bb)]
    acc = torch.zeros(8, dtype=torch.float64, device=DEV)
    _, mse, nll, mae, tot = heads_losses(*gin, y.float().to(DEV), factor.float().to(DEV), inv_psi.float().to(DEV),
                                        c_nll=coeffs[0], c_mse=coeffs[1], acc=acc)
    tot.backward()
    assert abs(tot.item() - tot_r.item()) <= 3e-5 * abs(tot_r.item()) + 1e-4
    for a, b in zip(gin, ref_in):
        torch.testing.assert_close(a.grad.double().cpu(), b.grad, rtol=5e-4, atol=5e-5)
    a = acc.cpu()
    assert abs(a[0] / a[1] - mse_r.item()) < 1e-5 and a[3] == 1 and abs(a[4] / a[5] - tot_r.item()) < 1e-3 * abs(
        tot_r.item()) + 1e-3


@pytest.mark.parametrize("N,B,mode,H", [(100, 1, "reference", 64), (37, 1, "reference", 16), (128, 1, "reference", 128),
                                         (100, 2, "per_window", 32), (120, 3, "per_window", 64),
                                         (200, 1, "reference", 64)])
@pytest.mark.parametrize("coeffs", [(0.0, 1.0), (1.0, 100.0)])
def test_training_decoder_matches_fp64(N, B, mode, H, coeffs):
    """ops/losses.py heads_losses_train (one launch: heads, losses, metric sums, dh_T, head gradients; the
    register-resident kernel for N <= 128, the LDS-staged one above) against fp64 autograd of heads_losses."""
    from masters_thesis_amd.ops.losses import heads_losses, heads_losses_train

    torch.manual_seed(N + H)
    n = 30
    h = torch.randn(N, H, dtype=torch.float64) * 0.5
    wa, ba = torch.randn(1, H, dtype=torch.float64) * 0.1, torch.randn(1, dtype=torch.float64) * 0.1
    wb, bb = torch.randn(1, H, dtype=torch.float64) * 0.1, torch.ones(1, dtype=torch.float64)
    y = torch.randn(N, n, 4, dtype=torch.float64) * 0.02
    factor = torch.stack([torch.randn(B) * 0.01, torch.rand(B) * 0.002 + 0.001], -1).double()
    inv_psi = torch.rand(N, dtype=torch.float64) * 300 + 100
    ref_in = [t.clone().requires_grad_(True) for t in (h, wa, ba, wb, bb)]
    _, mse_r, nll_r, mae_r, tot_r = heads_losses(*ref_in, y, factor, inv_psi, batch_windows=B, nll_mode=mode,
                                                 c_nll=coeffs[0], c_mse=coeffs[1])
    tot_r.backward()
    d = lambda t: t.float().to(DEV)  # noqa: E731
    grads = [torch.zeros(H, device=DEV), torch.zeros(1, device=DEV), torch.zeros(H, device=DEV),
             torch.zeros(1, device=DEV)]
    acc = torch.zeros(8, dtype=torch.float64, device=DEV)
    res = heads_losses_train(d(h), d(wa).flatten(), d(ba), d(wb).flatten(), d(bb), d(y), d(factor), d(inv_psi),
                             batch_windows=B, want_nll=coeffs[0] != 0, nll_mode=mode, c_nll=coeffs[0],
                             c_mse=coeffs[1], acc=acc, grads=grads)
    assert res is not None
    out, dh = res
    torch.cuda.synchronize()
    o = out.double().cpu()
    assert abs(o[0] - mse_r.item()) <= 1e-5 * abs(mse_r.item())
    assert abs(o[2] - mae_r.item()) <= 1e-5 * abs(mae_r.item())
    if coeffs[0]:
        assert abs(o[1] - nll_r.item()) <= 2e-5 * abs(nll_r.item()) + 1e-3
    assert abs(o[3] - tot_r.item()) <= 3e-5 * abs(tot_r.item()) + 1e-3

    def close(a, b):
        err = (a.double().cpu() - b).abs().max().item()
        assert err <= 2e-4 * b.abs().max().item() + 1e-7, err

    close(dh, ref_in[0].grad)
    close(grads[0], ref_in[1].grad.flatten())
    close(grads[1], ref_in[2].grad)
    close(grads[2], ref_in[3].grad.flatten())
    close(grads[3], ref_in[4].grad)
    a = acc.cpu()
    assert a[3] == 1 and abs(a[0] / a[1] - mse_r.item()) <= 1e-5 * abs(mse_r.item())


# (37 windows of 5 x 6 x 3, B = 4): 20 blocks; (300 windows of 100 x 60 x 3, B = 64): 1,280 blocks, two-level arrival
@pytest.mark.parametrize("W,K,T,B,stop", [(37, 5, 6, 4, 33), (300, 100, 60, 64, 290)])
def test_gather_batch_kernel_and_cursor(W, K, T, B, stop):
    from masters_thesis_amd.data.datamodule import TensorBatchLoader

    X = torch.randn(W, K, T, 3, device=DEV)
    Y = torch.randn(W, K, 4, 4, device=DEV)
    Fc = torch.randn(W, 2, device=DEV)
    P = torch.randn(W, K, device=DEV)
    ld = TensorBatchLoader([X, Y, Fc, P], B, shuffle=True, seed=3, start=2, stop=stop)
    assert ld.supports_static()
    for epoch in (1, 2):
        nfull = ld.begin_epoch(epoch)
        idx = ld._epoch_idx
        for k in range(nfull):
            bufs = ld.gather_static()
            sel = idx[k * B:(k + 1) * B].to(DEV).long()
            for s, b in zip((X, Y, Fc, P), bufs):
                torch.testing.assert_close(b, s.index_select(0, sel), rtol=0, atol=0)
        assert int(ld._cursor.item()) == nfull and int(ld._arrive.abs().sum().item()) == 0
    tail = ld.tail_batch()
    assert tail is not None and tail[0].shape[0] == idx.numel() - B * nfull


def test_train_step_graph_matches_eager():
    """A captured train step (gather + fwd + bwd + clip/Adam in one graph) equals eager steps."""
    from masters_thesis_amd.data.datamodule import TensorBatchLoader
    from masters_thesis_amd.engine import Trainer
    from masters_thesis_amd.models import FinancialLstmCombined

    def run(graphs):
        torch.manual_seed(11)
        model = FinancialLstmCombined(dropout=0.0)
        W = 12
        g = torch.Generator().manual_seed(0)
        data = [torch.randn(W, 100, 60, 3, generator=g), torch.randn(W, 100, 30, 4, generator=g),
                torch.stack([torch.randn(W, generator=g) * 0.1, torch.rand(W, generator=g) + 0.2], -1),
                torch.rand(W, 100, generator=g) * 3 + 1]
        ld = TensorBatchLoader([d.to(DEV) for d in data], 1, shuffle=True, seed=0)
        tr = Trainer(gradient_clip_val=5.0, enable_progress_bar=False, enable_model_summary=False,
                     use_hip_graphs=graphs, matmul_precision="highest")
        tr._setup_env()
        tr._setup_model(model)
        tr._configure_optimizers(model)
        model.train()
        step = tr.make_train_stepper(ld)
        for _ in range(8):
            step()
        torch.cuda.synchronize()
        return tr.flat.data.clone(), model.train_acc.acc.clone()

    p_eager, acc_eager = run(False)
    p_graph, acc_graph = run(True)
    torch.testing.assert_close(p_graph, p_eager, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(acc_graph, acc_eager, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("B", [64, 8])
@pytest.mark.parametrize("mode", ["reference", "per_window"])
def test_grid_losses_match_single_workgroup(mode, B, monkeypatch):
    """N >= 512 (LG_MIN_N): the three-launch grid losses (csrc/losses.hip L1-L3) agree with the single-workgroup
    kernel."""
    from masters_thesis_amd.ops.losses import decoder_losses

    torch.manual_seed(5)
    K, n = 100, 30
    N = B * K
    ab = (torch.randn(N, 2) * 0.3 + torch.tensor([0.0, 1.0])).to(DEV)
    y = torch.randn(N, n, 4, device=DEV)
    factor = torch.stack([torch.randn(B) * 0.1, torch.rand(B) * 0.5 + 0.2], -1).to(DEV)
    inv_psi = (torch.rand(N) * 5 + 1).to(DEV)

    def run():
        a = ab.clone().requires_grad_(True)
        mse, nll, mae = decoder_losses(a, y, factor, inv_psi, batch_windows=B, nll_mode=mode)
        (mse * 0.7 + nll * 1.3).backward()
        return torch.stack([mse, nll, mae]).detach(), a.grad

    s_grid, g_grid = run()
    s_grid2, g_grid2 = run()
    assert torch.equal(s_grid, s_grid2) and torch.equal(g_grid, g_grid2)  # fixed-order sums
    monkeypatch.setenv("MTA_LOSSES_SINGLE", "1")
    s_one, g_one = run()
    torch.testing.assert_close(s_grid, s_one, rtol=2e-5, atol=1e-4)
    torch.testing.assert_close(g_grid, g_one, rtol=1e-4, atol=1e-4 * g_one.abs().max().item())


@pytest.mark.parametrize("B,H", [(64, 2048), (8, 512)])
def test_wide_heads_losses_grid_path(B, H):
    """N*H above the fused single-workgroup limit: grid-parallel heads forward / backward."""
    from masters_thesis_amd.ops.losses import heads_losses

    torch.manual_seed(9)
    N, n = 100 * B, 30
    h = torch.randn(N, H, dtype=torch.float64) * 0.1
    wa, ba = torch.randn(1, H, dtype=torch.float64) * 0.05, torch.randn(1, dtype=torch.float64) * 0.1
    wb, bb = torch.randn(1, H, dtype=torch.float64) * 0.05, torch.ones(1, dtype=torch.float64)
    y = torch.randn(N, n, 4, dtype=torch.float64)
    factor = torch.stack([torch.randn(B) * 0.1, torch.rand(B) * 0.5 + 0.2], -1).double()
    inv_psi = torch.rand(N, dtype=torch.float64) * 3 + 1
    ref_in = [t.clone().requires_grad_(True) for t in (h, wa, ba, wb, bb)]
    _, _, _, _, tot_r = heads_losses(*ref_in, y, factor, inv_psi, batch_windows=B, nll_mode="per_window",
                                     c_nll=1.0, c_mse=100.0)
    tot_r.backward()
    gin = [t.float().to(DEV).requires_grad_(True) for t in (h, wa, ba, wb, bb)]
    _, _, _, _, tot = heads_losses(*gin, y.float().to(DEV), factor.float().to(DEV), inv_psi.float().to(DEV),
                                   batch_windows=B, nll_mode="per_window", c_nll=1.0, c_mse=100.0)
    tot.backward()
    assert abs(tot.item() - tot_r.item()) <= 1e-4 * abs(tot_r.item())
    for a, b in zip(gin, ref_in):
        err = (a.grad.double().cpu() - b.grad).abs().max().item()
        assert err <= 1e-3 * b.grad.abs().max().item() + 1e-6, err


@pytest.mark.parametrize("prec,tol", [(0, 1e-5), (1, 2e-5), (2, 1e-2)])
@pytest.mark.parametrize("M,N,K,bkn", [(6000, 512, 128, False), (777, 64, 256, True), (960, 256, 3, False),
                                       (100, 5, 256, True), (33, 70, 45, False)])
def test_gemm_f32_matches_fp64(prec, tol, M, N, K, bkn):
    """csrc/gemm_f32.hip (the per-layer LSTM path's input projection / input gradient) vs fp64, with bias
    and mask epilogues, both B layouts and ragged edges."""
    from masters_thesis_amd.ops._lib import lib

    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(K, N, generator=g) if bkn else torch.randn(N, K, generator=g)
    bias = torch.randn(N, generator=g)
    mask = (torch.rand(M, N, generator=g) > 0.2).float() * 1.25
    ref = A.double() @ (B.double() if bkn else B.double().t())
    ref = (ref + bias.double()) * mask.double()
    C = torch.empty(M, N, device=DEV)
    lib().gemm_f32(prec, A.to(DEV), B.to(DEV), C, bias.to(DEV), mask.to(DEV), bkn)
    torch.cuda.synchronize()
    scale = (A.double().abs() @ (B.double().abs() if bkn else B.double().abs().t())).max().item()
    assert (C.double().cpu() - ref).abs().max().item() <= tol * scale


def test_per_layer_path_runs_no_library_gemm():
    """H=128 (per-layer kernels) and a non-fused layer-0 width: the input projections and input gradients are
    the hand-written MFMA GEMM, not hipBLASLt/rocBLAS (no Cijk_* kernel in the trace)."""
    from masters_thesis_amd.ops.lstm import lstm_last_hidden

    torch.manual_seed(3)
    x = torch.randn(100, 60, 8, device=DEV, requires_grad=True)
    ws = [w.to(DEV).requires_grad_(True) for w in _lstm_weights(8, 128, 2)]
    lstm_last_hidden(x, ws, 2, 0.2, True, "high").sum().backward()  # warm-up (library handles etc.)
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        lstm_last_hidden(x, ws, 2, 0.2, True, "high").sum().backward()
        torch.cuda.synchronize()
    names = [e.name for e in prof.events()]
    assert any("gemm_f32_kernel" in n for n in names), sorted(set(names))[:20]
    assert not any(n.startswith("Cijk") or "rocblas" in n.lower() for n in names), \
        [n for n in names if n.startswith("Cijk")][:5]
