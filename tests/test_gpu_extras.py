"""Numerics of the north-star extra kernels (GEMM / norms / RoPE attention) and encoders vs fp32 PyTorch."""
import math

import pytest
import torch
import torch.nn.functional as Fn

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _native():
    from masters_thesis_amd.ops import _lib

    assert _lib.lib(required=True) is not None


def _bf(x):
    return x.to(DEV, torch.bfloat16)


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("M,N,K", [(112, 256, 184), (6000, 384, 128), (64, 64, 32), (200, 136, 520), (2048, 2048, 200),
                                   (4104, 1032, 520), (4096, 1024, 136)])
def test_gemm_forward_epilogues(M, N, K):
    from masters_thesis_amd.ops import extras as X

    torch.manual_seed(0)
    A, W = torch.randn(M, K) * 0.5, torch.randn(N, K) * 0.1
    bias, res = torch.randn(N), torch.randn(M, N)
    Ab, Wb = _bf(A), _bf(W)
    ref_pre = Ab.float() @ Wb.float().t() + bias.to(DEV)
    pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    out = torch.empty(M, N, device=DEV)
    X.gemm(0, Ab, Wb, M, N, K, K, K, flags=X.EPI_BIAS | X.EPI_GELU | X.EPI_RESID, bias=bias.to(DEV),
           resid=res.to(DEV), aux_pre=pre, out_f32=out)
    assert _rel(pre.float(), ref_pre) < 5e-3
    assert _rel(out, Fn.gelu(ref_pre) + res.to(DEV)) < 2e-3


def test_gemm_input_grad_dgelu_and_weight_grad_split():
    from masters_thesis_amd.ops import extras as X

    torch.manual_seed(1)
    M, D, Din = 6000, 128, 96
    dY, W, Xa, pre = torch.randn(M, D), torch.randn(D, Din) * 0.1, torch.randn(M, Din), torch.randn(M, D)
    dYb, Wb, Xb, preb = _bf(dY), _bf(W), _bf(Xa), _bf(pre)
    # input grad: dX = dY W
    dX = torch.empty(M, Din, device=DEV)
    X.gemm(1, dYb, Wb, M, Din, D, D, Din, out_f32=dX)
    assert _rel(dX, dYb.float() @ Wb.float()) < 2e-3
    # input grad with GELU' epilogue (through W^T of a square layer)
    W2b = _bf(torch.randn(Din, D) * 0.1)  # a D -> Din layer: weight [out=Din][in=D]
    dpre = torch.empty(M, D, device=DEV, dtype=torch.bfloat16)
    dAct = torch.randn(M, Din)
    X.gemm(1, _bf(dAct), W2b, M, D, Din, Din, D, flags=X.EPI_DGELU, aux_in=preb, out_bf16=dpre)
    p = preb.float().requires_grad_(True)
    (g,) = torch.autograd.grad(Fn.gelu(p), p, _bf(dAct).float() @ W2b.float())
    assert _rel(dpre.float(), g) < 8e-3
    # weight grad with split-K, bias grad and an n_store narrower than the padded width
    gW = torch.ones(D, Din - 3, device=DEV)  # accumulates on top of existing grads
    gb = torch.ones(D, device=DEV)
    X.gemm(2, dYb, Xb, D, Din, M, D, Din, flags=X.EPI_ACCUM, out_f32=gW, ldc=Din - 3, n_store=Din - 3,
           ksplit=X.wgrad_split(D, Din, M), bias_grad=gb)
    ref = dYb.float().t() @ Xb.float()
    assert _rel(gW - 1, ref[:, :Din - 3]) < 2e-3
    assert _rel(gb - 1, dYb.float().sum(0)) < 2e-3


def _ran_kernel(fn, name):
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    return any(name in e.key for e in prof.key_averages())


def _ran_big(fn):
    """The 256 x 256 kernel ran."""
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    return any("gemm_big_kernel" in e.key for e in prof.key_averages())


# the 256 x 256 LDS-DMA kernel (csrc/gemm.hip, namespace big) in its three operand layouts, on ragged shapes (M, N not
# multiples of 256, K a multiple of 32 but not of 64, re-split K for the accumulating weight gradient), against an fp32
# PyTorch product and against the 128-tile path of the same call
@pytest.mark.parametrize("mode,M,N,K", [(0, 4000, 2056, 544), (0, 4096, 2048, 2048), (1, 4000, 2056, 544),
                                        (1, 6400, 2048, 2048), (2, 1032, 776, 4000), (2, 2048, 2048, 6400)])
def test_big_tile_gemm(mode, M, N, K):
    from masters_thesis_amd.ops import _lib
    from masters_thesis_amd.ops import extras as X

    C = _lib.lib()
    torch.manual_seed(mode * 7 + M)
    if mode == 0:
        A, B = _bf(torch.randn(M, K) * 0.5), _bf(torch.randn(N, K) * 0.1)
        bias, res = torch.randn(N, device=DEV), torch.randn(M, N, device=DEV)
        ref_pre = A.float() @ B.float().t() + bias
        outs = []
        for big in (1, 0):
            C.gemm_set_big(big)
            pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            out = torch.empty(M, N, device=DEV)
            fn = lambda: X.gemm(0, A, B, M, N, K, K, K, flags=X.EPI_BIAS | X.EPI_GELU | X.EPI_RESID,  # noqa: E731
                                bias=bias, resid=res, aux_pre=pre, out_f32=out)
            assert _ran_big(fn) == bool(big)
            assert _rel(pre.float(), ref_pre) < 5e-3
            assert _rel(out, Fn.gelu(ref_pre) + res) < 2e-3
            outs.append(out.clone())
    elif mode == 1:
        A, B = _bf(torch.randn(M, K)), _bf(torch.randn(K, N) * 0.1)  # dY [M][K], W [K=out][N=in]
        pre = _bf(torch.randn(M, N))
        p = pre.float().requires_grad_(True)
        (ref,) = torch.autograd.grad(Fn.gelu(p), p, A.float() @ B.float())
        outs = []
        for big in (1, 0):
            C.gemm_set_big(big)
            out = torch.empty(M, N, device=DEV)
            fn = lambda: X.gemm(1, A, B, M, N, K, K, N, flags=X.EPI_DGELU, aux_in=pre, out_f32=out)  # noqa: E731
            assert _ran_big(fn) == bool(big)
            assert _rel(out, ref) < 3e-3
            outs.append(out.clone())
    else:
        A, B = _bf(torch.randn(K, M)), _bf(torch.randn(K, N))  # dY [tokens][M], X [tokens][N]
        ref = A.float().t() @ B.float()
        outs = []
        for big in (1, 0):
            C.gemm_set_big(big)
            gw = torch.ones(M, N, device=DEV)
            gb = torch.ones(M, device=DEV)
            fn = lambda: X.gemm(2, A, B, M, N, K, M, N, flags=X.EPI_ACCUM, out_f32=gw, ldc=N, n_store=N,  # noqa: E731
                                ksplit=X.wgrad_split(M, N, K), bias_grad=gb)
            assert _ran_big(fn) == bool(big)
            assert _rel(gw - 1, ref) < 2e-3
            assert _rel(gb - 1, A.float().sum(0)) < 2e-3
            outs.append(gw.clone())
    C.gemm_set_big(-1)
    assert _rel(outs[0], outs[1]) < 2e-3


# the transformer's small weight gradients (dY^T X: out <= 512 x 512, K = tokens) on the register-staged tiles, split-K
# (atomics) and unsplit (deterministic mode), against fp32 PyTorch (the 128 x 128 LDS-DMA form measured slower and
# was removed, profiles/r3_gemm_mid_negative.txt)
@pytest.mark.parametrize("M,N,K,ks", [(512, 128, 6272, 16), (128, 512, 6272, 16), (384, 128, 6272, 1), (200, 136, 4000, 8)])
def test_small_weight_grad(M, N, K, ks):
    from masters_thesis_amd.ops import extras as X

    torch.manual_seed(M + N)
    A, B = _bf(torch.randn(K, M)), _bf(torch.randn(K, N))
    ref = A.float().t() @ B.float()
    gw = torch.ones(M, N, device=DEV)
    gb = torch.ones(M, device=DEV)
    X.gemm(2, A, B, M, N, K, M, N, flags=X.EPI_ACCUM, out_f32=gw, ldc=N, n_store=N, ksplit=ks, bias_grad=gb)
    assert _rel(gw - 1, ref) < 2e-3
    assert _rel(gb - 1, A.float().sum(0)) < 2e-3


@pytest.mark.parametrize("split", [True, False])
def test_grouped_weight_grads(split):
    """Weight gradients queued over a backward (``group=True``) and launched together by gemm_group_flush: both
    operand layouts (dY^T X on [K][rows] operands, and the k-contiguous NN form), problems of different shapes in
    one launch, split-K (fp32 atomics) and unsplit (deterministic mode), accumulated onto existing values, bias
    gradients included -- against fp32 PyTorch."""
    from masters_thesis_amd.ops import extras as X

    torch.manual_seed(7)
    K = 6272
    shapes = [(384, 128), (128, 128), (512, 128), (128, 512), (128, 8)]
    probs = []
    for i, (M, N) in enumerate(shapes):
        for nn in (False, True):
            if nn:
                A, B = _bf(torch.randn(M, K)), _bf(torch.randn(N, K))  # k-contiguous images
                ref = A.float() @ B.float().t()
                bsum = None
            else:
                A, B = _bf(torch.randn(K, M)), _bf(torch.randn(K, N))
                ref = A.float().t() @ B.float()
                bsum = A.float().sum(0)
            out = torch.randn(M, N, device=DEV)
            bg = torch.randn(M, device=DEV) if bsum is not None else None
            probs.append((nn, A, B, M, N, out, out.clone(), ref, bg, None if bg is None else bg.clone(), bsum))
    for nn, A, B, M, N, out, _, _, bg, _, _ in probs:
        ks = X.wgrad_split(M, N, K) if split else 1
        if nn:
            X.gemm(0, A, B, M, N, K, K, K, flags=X.EPI_ACCUM, out_f32=out, ldc=N, n_store=N, ksplit=ks, group=True)
        else:
            X.gemm(2, A, B, M, N, K, M, N, flags=X.EPI_ACCUM, out_f32=out, ldc=N, n_store=N, ksplit=ks, bias_grad=bg,
                   group=True)
    X.gemm_group_flush()
    torch.cuda.synchronize()
    for nn, A, B, M, N, out, out0, ref, bg, bg0, bsum in probs:
        assert _rel(out - out0, ref) < 2e-3, (nn, M, N)
        if bg is not None:
            assert _rel(bg - bg0, bsum) < 2e-3, (M, N)


@pytest.mark.parametrize("rms", [False, True])
@pytest.mark.parametrize("D", [128, 256, 1024, 1536, 2048])
def test_norm_forward_backward(rms, D):
    from masters_thesis_amd.ops import _lib
    from masters_thesis_amd.ops.extras import LN_EPS, RMS_EPS

    C = _lib.lib()
    torch.manual_seed(2)
    M = 301 if D < 1024 else 2600  # wide rows: > the 1,024-workgroup grid, so workgroups stride over rows
    x = (torch.randn(M, D) * 2 + 0.5).to(DEV)
    g, b = (torch.rand(D) + 0.5).to(DEV), torch.randn(D).to(DEV)
    dy = torch.randn(M, D).to(DEV)
    pre = _bf(torch.randn(M, D))
    dres = torch.randn(M, D).to(DEV)
    eps = RMS_EPS if rms else LN_EPS
    yb = torch.empty(M, D, device=DEV, dtype=torch.bfloat16)
    yf = torch.empty(M, D, device=DEV)
    mean = None if rms else torch.empty(M, device=DEV)
    rstd = torch.empty(M, device=DEV)
    C.norm(False, x, D, M, D, rms, eps, g, None if rms else b, yb, yf, mean, rstd, None, 0.0, None, None, None, None,
           None, None, None)
    xr, gr, br = x.clone().requires_grad_(True), g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    ref = Fn.rms_norm(xr, (D,), gr, eps) if rms else Fn.layer_norm(xr, (D,), gr, br, eps)
    assert _rel(yf, ref) < 1e-5 and _rel(yb.float(), ref) < 5e-3
    dxf = torch.empty(M, D, device=DEV)
    dgam = torch.zeros(D, device=DEV)
    dbet = torch.zeros(D, device=DEV)
    C.norm(True, x, D, M, D, rms, eps, g, None if rms else b, None, None, mean, rstd, None, 0.0, dy, dres, None, None,
           dxf, dgam, None if rms else dbet)
    gx, gg, gb = torch.autograd.grad(ref, (xr, gr, br), dy, allow_unused=True)
    assert _rel(dxf - dres, gx) < 1e-4
    assert _rel(dgam, gg) < 1e-4
    if not rms:
        assert _rel(dbet, gb) < 1e-4
    # GELU' fusion (D = 1024 / 2048: the branch-free wide backward, with its parameter partials)
    dxb = torch.empty(M, D, device=DEV, dtype=torch.bfloat16)
    dgam2 = torch.zeros(D, device=DEV)
    dbet2 = torch.zeros(D, device=DEV)
    C.norm(True, x, D, M, D, rms, eps, g, None if rms else b, None, None, mean, rstd, None, 0.0, dy, None, pre, dxb,
           None, dgam2, None if rms else dbet2)
    p = pre.float().requires_grad_(True)
    (gp,) = torch.autograd.grad(Fn.gelu(p), p, gx)
    assert _rel(dxb.float(), gp) < 8e-3
    assert _rel(dgam2, gg) < 1e-4
    if not rms:
        assert _rel(dbet2, gb) < 1e-4
    # the parameter reduction is fixed-order (per-block partial rows, xor-tree + wave-order column sums): bit-identical reruns
    dgam3 = torch.zeros(D, device=DEV)
    C.norm(True, x, D, M, D, rms, eps, g, None if rms else b, None, None, mean, rstd, None, 0.0, dy, None, pre, dxb,
           None, dgam3, None)
    assert torch.equal(dgam2, dgam3)


@pytest.mark.parametrize("rms", [False, True])
@pytest.mark.parametrize("D", [1024, 2048])
def test_norm_gelu_on_load(rms, D):
    """The bf16 MLP's norm pair with the GELU applied on load (gelu_x: x is the bf16 pre-activation, the normalised row
    is gelu(x)): forward against fp32 PyTorch LayerNorm / RMSNorm of gelu(pre), backward (dx through the norm and the
    GELU, dgamma, dbeta) against autograd of the same fp32 composition."""
    from masters_thesis_amd.ops import _lib
    from masters_thesis_amd.ops.extras import LN_EPS, RMS_EPS

    C = _lib.lib()
    torch.manual_seed(5)
    M = 2600
    pre = _bf(torch.randn(M, D) * 1.5)
    g, b = (torch.rand(D) + 0.5).to(DEV), torch.randn(D).to(DEV)
    dy = torch.randn(M, D).to(DEV)
    eps = RMS_EPS if rms else LN_EPS
    yb = torch.empty(M, D, device=DEV, dtype=torch.bfloat16)
    yf = torch.empty(M, D, device=DEV)
    mean = None if rms else torch.empty(M, device=DEV)
    rstd = torch.empty(M, device=DEV)
    C.norm(False, pre, D, M, D, rms, eps, g, None if rms else b, yb, yf, mean, rstd, None, 0.0, None, None, None, None,
           None, None, None, gelu_x=True)
    p = pre.float().requires_grad_(True)
    gr, br = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    act = Fn.gelu(p)
    ref = Fn.rms_norm(act, (D,), gr, eps) if rms else Fn.layer_norm(act, (D,), gr, br, eps)
    assert _rel(yf, ref) < 1e-5 and _rel(yb.float(), ref) < 5e-3
    dxb = torch.empty(M, D, device=DEV, dtype=torch.bfloat16)
    dgam = torch.zeros(D, device=DEV)
    dbet = torch.zeros(D, device=DEV)
    C.norm(True, pre, D, M, D, rms, eps, g, None if rms else b, None, None, mean, rstd, None, 0.0, dy, None, pre, dxb,
           None, dgam, None if rms else dbet, gelu_x=True)
    gp, gg, gb = torch.autograd.grad(ref, (p, gr, br), dy, allow_unused=True)
    assert _rel(dxb.float(), gp) < 8e-3
    assert _rel(dgam, gg) < 1e-4
    if not rms:
        assert _rel(dbet, gb) < 1e-4


@pytest.mark.parametrize("norm", ["layernorm", "rmsnorm"])
def test_mlp_fused_heads_match_unfused(norm):
    """The alpha / beta heads fused into the MLP's last norm kernels (ops.extras.mlp_encode_heads: ab from the
    normalised rows in-kernel, dy = d_alpha wa + d_beta wb formed in the norm backward, head-weight gradients from h
    recomputed there) against the same bf16 encoder returning h followed by an fp32 addmm and autograd: ab, every
    encoder gradient and the four head gradients.  N = 300 exercises the 16-row padding (pad rows: zero d(ab))."""
    from masters_thesis_amd.models.extras import MLPEncoder
    from masters_thesis_amd.ops import extras as X

    torch.manual_seed(7)
    N, T, F, H, L = 300, 60, 3, 1024, 2
    enc = MLPEncoder(F, T, H, L, 0.0, norm).to(DEV)
    x = torch.randn(N, T, F, device=DEV)
    heads = [torch.randn(1, H, device=DEV) * 0.03, torch.randn(1, device=DEV) * 0.1,
             torch.randn(1, H, device=DEV) * 0.03, torch.randn(1, device=DEV) * 0.1]
    heads = [t.requires_grad_(True) for t in heads]
    G = torch.randn(N, 2, device=DEV)
    params = enc.flat_params()
    assert X.mlp_heads_fusable(x, params, L, norm, "medium")
    runs = []
    for fused in (True, False):
        for t in list(params) + heads:
            t.grad = None
        if fused:
            ab = X.mlp_encode_heads(x, params, enc.seeds, L, norm, 0.0, True, "medium", heads)
        else:
            h = X.mlp_encode(x, params, enc.seeds, L, norm, 0.0, True, "medium")
            ab = torch.addmm(torch.cat([heads[1], heads[3]]), h, torch.cat([heads[0], heads[2]], 0).t())
        (ab * G).sum().backward()
        torch.cuda.synchronize()
        runs.append((ab.detach().clone(), [t.grad.detach().clone() for t in list(params) + heads]))
    (ab_f, g_f), (ab_u, g_u) = runs
    assert _rel(ab_f, ab_u) < 1e-5
    for k, (a, b) in enumerate(zip(g_f, g_u)):
        assert _rel(a, b) < (1e-5 if k >= len(params) else 2e-3), (k, _rel(a, b))


@pytest.mark.parametrize("T,heads,hd", [(60, 4, 32), (64, 2, 64), (17, 3, 32)])
def test_attention_forward_backward(T, heads, hd):
    from masters_thesis_amd.ops import _lib
    from masters_thesis_amd.ops.extras import ROPE_BASE, attention_reference

    C = _lib.lib()
    torch.manual_seed(3)
    N, d = 24, heads * hd
    qkv = _bf(torch.randn(N * T, 3 * d))
    out = torch.empty(N * T, d, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(N * heads * 64, device=DEV)
    C.attention(False, qkv, out, lse, None, None, N, T, d, heads, ROPE_BASE)
    q = qkv.float().view(N, T, 3 * d).requires_grad_(True)
    ref = attention_reference(q, heads)
    assert _rel(out.float().view(N, T, d), ref) < 1e-2
    dout = _bf(torch.randn(N * T, d))
    dqkv = torch.empty(N * T, 3 * d, device=DEV, dtype=torch.bfloat16)
    C.attention(True, qkv, out, lse, dout, dqkv, N, T, d, heads, ROPE_BASE)
    (gq,) = torch.autograd.grad(ref, q, dout.float().view(N, T, d))
    gq = gq.view(N * T, 3 * d)
    for part in range(3):
        sl = slice(part * d, (part + 1) * d)
        assert _rel(dqkv.float()[:, sl], gq[:, sl]) < 2.5e-2, part


def _encoder_parity(model_cls, kw, tol_h, tol_g):
    torch.manual_seed(5)
    cpu = model_cls(**kw)
    gpu = model_cls(**kw)
    gpu.load_state_dict(cpu.state_dict())
    gpu = gpu.to(DEV)
    x = torch.randn(100, 60, 3) * 0.8
    cpu.train()
    gpu.train()
    h_ref = cpu.encode(x)
    h = gpu.encode(x.to(DEV))
    w = torch.randn_like(h_ref)
    (h_ref * w).sum().backward()
    (h * w.to(DEV)).sum().backward()
    assert _rel(h.cpu(), h_ref.detach()) < tol_h
    for (n, p_ref), (_, p) in zip(cpu.encoder.named_parameters(), gpu.encoder.named_parameters()):
        assert p.grad is not None, n
        e = _rel(p.grad.cpu(), p_ref.grad)
        assert e < tol_g, (n, e)


@pytest.mark.parametrize("norm", ["layernorm", "rmsnorm"])
def test_mlp_encoder_matches_fp32_reference(norm):
    from masters_thesis_amd.models.extras import FinancialMlpMse

    _encoder_parity(FinancialMlpMse, dict(hidden_size=256, num_layers=3, dropout=0.0, norm=norm), 2e-2, 5e-2)


def test_transformer_encoder_matches_fp32_reference():
    from masters_thesis_amd.models.extras import FinancialTransformerMse

    _encoder_parity(FinancialTransformerMse, dict(hidden_size=128, num_layers=2, num_heads=4, dropout=0.0), 3e-2, 8e-2)


@pytest.mark.parametrize("M", [6272, 2400 + 40])
def test_tr_attn_dx_matches_reference(M):
    """csrc/tr_attn.hip tr_attn_dx: d(xn) = dqkv Wqkv (Wqkv^T fragment-major image) and the RMSNorm1 backward with
    the residual gradient, against fp32 PyTorch autograd of rms_norm on the same bf16 operands: dX (fp32 and bf16)
    and dg1 (summed from the deferred norm slot at norm_flush).  M = 2,440: a partial last 64-row tile."""
    import torch.nn.functional as Fn

    from masters_thesis_amd.ops._lib import lib

    C = lib()
    torch.manual_seed(11)
    dqkv = _bf(torch.randn(M, 384) * 0.5)
    wqkv = torch.randn(384, 128, device=DEV) * 0.05
    x = torch.randn(M, 128, device=DEV)
    g1 = 1.0 + 0.1 * torch.randn(128, device=DEV)
    dx1 = torch.randn(M, 128, device=DEV)
    r1 = torch.rsqrt(x.pow(2).mean(-1) + 1e-6)
    wt = torch.empty(128, 384, device=DEV, dtype=torch.bfloat16)
    C.frag_pack([wqkv], [wt], [True])
    dx = torch.empty(M, 128, device=DEV)
    dxb = torch.empty(M, 128, device=DEV, dtype=torch.bfloat16)
    dg = torch.full((128,), 0.5, device=DEV)
    C.tr_attn_dx(dqkv, wt, x, r1, g1, dx1, dx, dxb, dg)
    C.norm_flush()
    torch.cuda.synchronize()
    dxn = dqkv.float() @ wqkv.bfloat16().float()
    xr = x.clone().requires_grad_(True)
    gr = g1.clone().requires_grad_(True)
    y = Fn.rms_norm(xr, (128,), gr, 1e-6)
    y.backward(dxn)
    ref = xr.grad + dx1
    assert _rel(dx, ref) < 1e-4
    assert _rel(dxb.float(), ref) < 1e-2
    assert _rel(dg - 0.5, gr.grad) < 1e-4


@pytest.mark.parametrize("dropout,N,T", [(0.0, 100, 60), (0.2, 37, 60), (0.0, 20, 33), (0.2, 305, 33), (0.0, 600, 33)])
def test_fused_transformer_ffn_matches_unfused(dropout, N, T):
    """csrc/tr_ffn.hip (the FFN half of every block in one launch forward and one backward, plus split-K weight
    gradients) and csrc/tr_attn.hip (the attention half forward in one launch) against the unfused kernel chain on the
    same inputs, seeds and weights: encoder output and every parameter gradient, plus the fp32 PyTorch reference
    without dropout.  N = 37: M = 40 x 60 rows, a partial 32-row workgroup at the end; T = 33: padded key masking.
    N = 305 / 600 at T = 33: more 32-row tiles than CUs (the persistent FFN kernels walk 2-3 tiles per workgroup, the
    last one partial) and, at 600, weight-gradient K >= 16,384 (the grouped launches on 128 x 128 tiles)."""
    from masters_thesis_amd.models.extras import FinancialTransformerMse
    from masters_thesis_amd.ops import extras as X

    torch.manual_seed(3)
    m = FinancialTransformerMse(hidden_size=128, num_layers=2, num_heads=4, dropout=dropout).to(DEV)
    enc = m.encoder
    params = list(enc.flat_params()) if hasattr(enc, "flat_params") else [p for p in enc.parameters()]
    x = torch.randn(N, T, 3, device=DEV)
    seeds0 = torch.randint(0, 2 ** 62, (8,), device=DEV, dtype=torch.int64)
    outs, grads = [], []
    prev = X._TR_FFN[0], X._TR_ATTN[0], X._TR_WGRAD_NN[0]
    try:
        # fused with the FFN weight gradients on transposed (NN) operands, fused, unfused
        for fused, nn in ((True, True), (True, False), (False, False)):
            X.set_transformer_ffn_fused(fused)
            X.set_transformer_attn_fused(fused)
            X.set_transformer_wgrad_nn(nn)
            fn = lambda: X.transformer_encode(x, params, seeds0.clone(), 2, 4, dropout, False)  # noqa: E731
            assert _ran_kernel(fn, "tr_ffn_fwd_kernel") == fused
            assert _ran_kernel(fn, "tr_attn_fwd_kernel") == fused
            for p in params:
                p.grad = None
            seeds = seeds0.clone()
            h = X.transformer_encode(x, params, seeds, 2, 4, dropout, True)
            g = torch.randn(h.shape, device=DEV, generator=torch.Generator(device=DEV).manual_seed(5))
            # the fused attention half's backward: dO = dX1 Wo inside the attention backward, d(xn) = dqkv Wqkv with
            # the RMSNorm1 backward in tr_attn_dx; every weight gradient in the grouped launches
            with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
                h.backward(g)
                torch.cuda.synchronize()
            names = {e.key for e in prof.key_averages()}
            assert any("tr_attn_dx_kernel" in n for n in names) == fused, sorted(names)
            assert any("gemm_group_kernel" in n for n in names), sorted(names)
            outs.append(h.detach().clone())
            grads.append([p.grad.detach().clone() for p in params])
    finally:
        X.set_transformer_ffn_fused(prev[0])
        X.set_transformer_attn_fused(prev[1])
        X.set_transformer_wgrad_nn(prev[2])
    for i in (0, 1):
        assert _rel(outs[i], outs[2]) < 2e-3
        for a, b in zip(grads[i], grads[2]):
            assert _rel(a, b) < 5e-3
    if dropout == 0.0:
        with torch.no_grad():
            ref = X.transformer_reference(x.double(), [p.double() for p in params], 2, 4, 0.0, False)
        assert _rel(outs[0], ref) < 3e-2


def test_extras_dropout_train_vs_eval_and_finite_grads():
    from masters_thesis_amd.models.extras import FinancialMlpCombined, FinancialTransformerCombined

    batch = (torch.randn(1, 100, 60, 3, device=DEV), torch.randn(1, 100, 30, 4, device=DEV),
             torch.tensor([[0.05, 0.4]], device=DEV), torch.rand(1, 100, device=DEV) + 1)
    for cls, kw in ((FinancialMlpCombined, dict(hidden_size=128, num_layers=3, dropout=0.3)),
                    (FinancialTransformerCombined, dict(hidden_size=64, num_layers=2, num_heads=2, dropout=0.3))):
        torch.manual_seed(0)
        m = cls(**kw).to(DEV)
        m.eval()
        with torch.no_grad():
            h_eval = m.encode(batch[0][0])
        m.train()
        h1 = m.encode(batch[0][0])
        h2 = m.encode(batch[0][0])
        assert not torch.allclose(h1, h_eval) and not torch.allclose(h1, h2)  # fresh mask per call
        loss = m.training_step(batch, 0)
        loss.backward()
        assert all(torch.isfinite(p.grad).all() for p in m.parameters() if p.grad is not None)


@pytest.mark.parametrize("arch", ["mlp", "transformer"])
def test_extras_train_through_trainer_graph(arch):
    """The extras encoders through the Trainer's captured training step (graph warm-up, capture, replays) with their
    fused step (one-launch decoder, models/extras.py fused_training_step): captured and replayed, training finite."""
    from masters_thesis_amd.data.datamodule import TensorBatchLoader
    from masters_thesis_amd.engine import Trainer
    from masters_thesis_amd.models import get_model_class

    g = torch.Generator().manual_seed(0)
    W = 6
    data = [torch.randn(W, 100, 60, 3, generator=g), torch.randn(W, 100, 30, 4, generator=g) * 0.01,
            torch.stack([torch.randn(W, generator=g) * 0.01, torch.rand(W, generator=g) * 1e-3 + 1e-4], -1),
            torch.rand(W, 100, generator=g) * 3 + 1]
    cls = get_model_class("FinancialLstmCombined", arch)
    kw = dict(input_size=3, hidden_size=128 if arch == "transformer" else 256, num_layers=2, dropout=0.1,
              learning_rate=1e-4)
    if arch == "transformer":
        kw.update(num_heads=4, mlp_ratio=4)
    model = cls(**kw)
    tr = Trainer(gradient_clip_val=5.0, enable_progress_bar=False, enable_model_summary=False, use_hip_graphs=True,
                 precision="bf16-mixed")
    tr._setup_env()
    tr._setup_model(model)
    tr._configure_optimizers(model)
    model.train()
    assert model.fused_step_supported([t[:1].to(DEV) for t in data])  # the loader's one-window batches
    step = tr.make_train_stepper(TensorBatchLoader([t.to(DEV) for t in data], 1, shuffle=True, seed=0))
    for _ in range(8):
        loss = step()
    torch.cuda.synchronize()
    assert torch.isfinite(tr.flat.data).all() and torch.isfinite(loss).all()
    assert tr._graphs  # the step was captured and replayed


@pytest.mark.parametrize("batch", [1, 32])
def test_mlp_grad_producers_match_accumulating_path(batch, monkeypatch):
    """Big MLP weight gradients as optimizer gradient PRODUCERS (csrc/gemm.hip mta_gemm_grad_producer: the split-K
    reduce overwrites the flat-gradient range and writes the clip-norm partials; the fused update skips re-reading and
    zeroing it) against the accumulate + zero path, through the Trainer's captured steps with clipping active: the
    parameter trajectories agree and the producers actually ran.  batch 1: K = 104 tokens, the fallback (zero-fill +
    accumulating GEMM + partials launch); batch 32: K = 3,200, the 256 x 256 kernel's fp32-slab split-K reduce."""
    from masters_thesis_amd.data.datamodule import TensorBatchLoader
    from masters_thesis_amd.engine import Trainer
    from masters_thesis_amd.models import get_model_class

    g = torch.Generator().manual_seed(0)
    W = 64
    data = [torch.randn(W, 100, 60, 3, generator=g), torch.randn(W, 100, 30, 4, generator=g) * 0.01,
            torch.stack([torch.randn(W, generator=g) * 0.01, torch.rand(W, generator=g) * 1e-3 + 1e-4], -1),
            torch.rand(W, 100, generator=g) * 3 + 1]
    outs, init, grads1, norms1 = [], None, [], []
    for prod in ("1", "0"):
        monkeypatch.setenv("MTA_OPTIM_PRODUCERS", prod)
        torch.manual_seed(1)
        model = get_model_class("FinancialLstmMse", "mlp")(input_size=3, hidden_size=1024, num_layers=3, dropout=0.0,
                                                             learning_rate=1e-3)
        tr = Trainer(gradient_clip_val=0.05, enable_progress_bar=False, enable_model_summary=False,
                     use_hip_graphs=True, precision="bf16-mixed")
        tr._setup_env()
        tr._setup_model(model)
        tr._configure_optimizers(model)
        init = tr.flat.data.detach().clone()
        model.train()
        opt_step = tr.optimizer.step

        def step_and_snapshot(max_norm=0.0, grad_scale=1.0, zero_grad=False, _opt_step=opt_step, _tr=tr, **kw):
            first = len(grads1) < len(outs) + 1
            if first:
                torch.cuda.synchronize()
                grads1.append(_tr.flat.grad.detach().clone())
            _opt_step(max_norm, grad_scale, zero_grad, **kw)
            if first:
                norms1.append(float(_tr.optimizer.grad_norm.item()))

        tr.optimizer.step = step_and_snapshot
        step = tr.make_train_stepper(TensorBatchLoader([t.to(DEV) for t in data], batch, shuffle=True, seed=0))
        for _ in range(10):
            step()
        torch.cuda.synchronize()
        outs.append(tr.flat.data.detach().clone())
        if prod == "1":
            assert tr.optimizer.ext_parts.abs().sum().item() > 0, "no gradient producer ran"
        assert tr.optimizer.nonfinite.item() == 0
    # the sharp check: step 1's flat gradient and clip norm (what the optimizer consumes) agree at fp32 precision.
    # Both paths write the same bf16-input products; they differ only in the order split-K partials are summed (the
    # producer's slab reduce vs the paired launch's f32 atomics), ~1e-7 relative per element
    rel = ((grads1[0] - grads1[1]).norm() / grads1[1].norm()).item()
    nrel = abs(norms1[0] - norms1[1]) / norms1[1]
    assert rel <= 1e-5, rel
    assert nrel <= 1e-5, norms1
    # the trajectory (a smoke): Adam turns a near-zero gradient's sign noise into a full lr-sized step, so compare
    # against the distance the parameters moved
    moved = (outs[1] - init).norm().item()
    diff = (outs[0] - outs[1])
    assert diff.norm().item() < 2e-3 * moved, (diff.norm().item(), moved)
    assert diff.abs().max().item() < 2e-4, diff.abs().max().item()


# (6400, 2048, *): above 2^31 MACs both products run on transposed copies through the NN kernel (csrc/gemm.hip
# to_nn); 2048 pairs them in one launch, 1032 gives the two different tile configurations (separate launches)
@pytest.mark.parametrize("M,D,Din", [(6720, 128, 512), (6720, 384, 128), (304, 64, 72), (6400, 2048, 2048),
                                     (6400, 2048, 1032)])
def test_paired_weight_and_input_grad_gemms(M, D, Din):
    """A deferred weight-gradient GEMM runs together with the next (input-gradient) GEMM in one paired launch:
    same results as two launches (split-K sums compared with a tolerance, the input gradient exactly)."""
    from masters_thesis_amd.ops import extras as X

    g = torch.Generator().manual_seed(M + D)
    dY = _bf(torch.randn(M, D, generator=g))
    Xa = _bf(torch.randn(M, Din, generator=g))
    W = _bf(torch.randn(D, Din, generator=g) * 0.1)
    outs = []
    for defer in (False, True):
        gw = torch.zeros(D, Din, device=DEV)
        gb = torch.zeros(D, device=DEV)
        dx = torch.empty(M, Din, device=DEV)
        X.gemm(2, dY, Xa, D, Din, M, D, Din, flags=X.EPI_ACCUM, out_f32=gw, ldc=Din,
               ksplit=X.wgrad_split(D, Din, M), bias_grad=gb, defer=defer)
        X.gemm(1, dY, W, M, Din, D, D, Din, out_f32=dx)
        X.gemm_flush()
        torch.cuda.synchronize()
        outs.append((gw, gb, dx))
    (gw0, gb0, dx0), (gw1, gb1, dx1) = outs
    torch.testing.assert_close(dx1, dx0, rtol=0, atol=0)
    torch.testing.assert_close(gw1, gw0, rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(gb1, gb0, rtol=1e-5, atol=1e-3)
    ref = dY.double().t() @ Xa.double()
    assert _rel(gw1, ref) < 1e-5
    assert _rel(gb1, dY.double().sum(0)) < 1e-5
    assert _rel(dx1, dY.double() @ W.double()) < 1e-5


def test_gemm_dropout_mask_forward_backward_consistent():
    """The GEMM-epilogue dropout (pair hash, 16-bit uniform) keeps 1-p of the elements and the backward DGELU
    epilogue zeroes exactly the elements the forward GELU epilogue dropped (same seed, same (row, col))."""
    from masters_thesis_amd.ops import extras as X

    M, N, K, p = 1024, 256, 64, 0.1
    g = torch.Generator().manual_seed(1)
    A = _bf(torch.randn(M, K, generator=g))
    W = _bf(torch.randn(N, K, generator=g) * 0.2)
    bias = torch.full((N,), 3.0, device=DEV)  # GELU(v) > 0 everywhere: zeros come from the mask only
    seed = torch.tensor([0x1234_5678_9ABC], dtype=torch.int64, device=DEV)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    X.gemm(0, A, W, M, N, K, K, K, flags=X.EPI_BIAS | X.EPI_GELU | X.EPI_DROPOUT, bias=bias, seed=seed, drop_p=p,
           out_bf16=out, aux_pre=pre)
    # backward: dPre = (dOut W2 ...) here dOut = ones via A2 = identity-like product of ones
    ones_a = _bf(torch.ones(M, 8))
    ones_b = _bf(torch.ones(8, N) / 8)  # [K][N] layout of mode 1: dY (M x 8) . B (8 x N) = ones
    dpre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    X.gemm(1, ones_a, ones_b, M, N, 8, 8, N, flags=X.EPI_DGELU | X.EPI_DROPOUT, aux_in=pre, seed=seed, drop_p=p,
           out_bf16=dpre)
    torch.cuda.synchronize()
    kept_f = out.float() != 0
    kept_b = dpre.float() != 0
    assert torch.equal(kept_f, kept_b)
    frac = kept_f.float().mean().item()
    assert abs(frac - (1 - p)) < 0.01, frac


def test_extras_deterministic_mode_bit_identical_at_batch_64():
    """Trainer(deterministic=True) with an extras encoder at B = 64 windows (N = 6,400 sequences: the wide-head
    backward takes its grid path): no split-K GEMM atomics and block-ordered head-parameter partials
    (csrc/losses.hip heads_part_reduce_kernel), so two runs give bit-identical parameters."""
    from masters_thesis_amd.data.datamodule import TensorBatchLoader
    from masters_thesis_amd.engine import Trainer
    from masters_thesis_amd.models import get_model_class
    from masters_thesis_amd.ops import extras as X
    from masters_thesis_amd.ops import losses as L
    from masters_thesis_amd.ops import lstm as op

    g = torch.Generator().manual_seed(0)
    W = 128
    data = [torch.randn(W, 100, 60, 3, generator=g), torch.randn(W, 100, 30, 4, generator=g) * 0.01,
            torch.stack([torch.randn(W, generator=g) * 0.01, torch.rand(W, generator=g) * 1e-3 + 1e-4], -1),
            torch.rand(W, 100, generator=g) * 3 + 1]
    dev_data = [t.to(DEV) for t in data]

    def run():
        torch.manual_seed(5)
        cls = get_model_class("FinancialLstmCombined", "mlp")
        model = cls(input_size=3, hidden_size=256, num_layers=2, dropout=0.1, learning_rate=1e-4)
        tr = Trainer(gradient_clip_val=5.0, enable_progress_bar=False, enable_model_summary=False,
                     use_hip_graphs=True, deterministic=True, precision="bf16-mixed")
        tr._setup_env()
        tr._setup_model(model)
        tr._configure_optimizers(model)
        model.train()
        step = tr.make_train_stepper(TensorBatchLoader(dev_data, 64, shuffle=True, seed=0))
        for _ in range(6):
            step()
        torch.cuda.synchronize()
        return tr.flat.data.clone()

    try:
        a, b = run(), run()
    finally:
        op.set_deterministic(False)
        X.set_deterministic(False)
        L.set_deterministic(False)
    assert torch.isfinite(a).all()
    assert torch.equal(a, b)


@pytest.mark.parametrize("arch", ["mlp", "transformer"])
def test_extras_honour_trainer_precision(arch, monkeypatch):
    """Under trainer precision 32-true the extras encoders run their fp32 HIP paths (_MlpEncoderF32Fn /
    _TransformerEncoderF32Fn -- asserted taken) within 1e-4 of the fp64 reference on the same weights; under bf16-mixed
    the bf16 HIP kernels (bf16 tolerance, not exact)."""
    from masters_thesis_amd.engine import Trainer
    from masters_thesis_amd.models import get_model_class
    from masters_thesis_amd.ops import extras as X

    fn = X._MlpEncoderF32Fn if arch == "mlp" else X._TransformerEncoderF32Fn
    calls = []
    orig = fn.apply
    monkeypatch.setattr(fn, "apply", lambda *a: calls.append(1) or orig(*a))
    torch.manual_seed(0)
    cls = get_model_class("FinancialLstmMse", arch)
    kw = dict(input_size=3, hidden_size=128, num_layers=2, dropout=0.0)
    if arch == "transformer":
        kw.update(num_heads=4)
    x = torch.randn(200, 60, 3, device=DEV)
    outs = {}
    for prec in ("32-true", "bf16-mixed"):
        model = cls(**kw)
        tr = Trainer(enable_progress_bar=False, enable_model_summary=False, precision=prec)
        tr._setup_env()
        tr._setup_model(model)
        model.eval()
        with torch.no_grad():
            h = model.encode(x)
            params = model.encoder.flat_params()
            if arch == "mlp":
                ref = X.mlp_reference(x.double(), [p.double() for p in params], 2, model.encoder.norm, 0.0, False)
            else:
                ref = X.transformer_reference(x.double(), [p.double() for p in params], 2, 4, 0.0, False)
        outs[prec] = (h.double() - ref).abs().max().item() / max(ref.abs().max().item(), 1.0)
    assert calls, "the 32-true fp32 HIP path was not taken"
    assert outs["32-true"] <= 1e-4, outs
    assert 1e-6 < outs["bf16-mixed"] <= 5e-2, outs


@pytest.mark.parametrize("prec,tol", [("high", 1e-4), ("highest", 2e-5)])
@pytest.mark.parametrize("heads", [4, 2])
def test_transformer_32true_hip_path_matches_fp64(prec, tol, heads, monkeypatch):
    """32-true transformer on HIP kernels (ops/extras.py _TransformerEncoderF32Fn: gemm_f32x GEMMs with fused bias /
    GELU / GELU' / residual epilogues, fp32 RMSNorm, fp32 RoPE attention csrc/attention_f32.hip at head dim 32 and 64)
    against the same encoder in fp64 on the CPU: forward and every parameter gradient.  The HIP path must be taken."""
    from masters_thesis_amd.models.extras import TransformerEncoder
    from masters_thesis_amd.ops import extras as X

    calls = []
    orig = X._TransformerEncoderF32Fn.apply
    monkeypatch.setattr(X._TransformerEncoderF32Fn, "apply", lambda *a: calls.append(1) or orig(*a))
    torch.manual_seed(0)
    enc = TransformerEncoder(3, 128, 2, heads, dropout=0.0).to(DEV)
    enc.precision = prec
    enc.train()
    x = torch.randn(40, 60, 3, device=DEV)
    R = torch.randn(40, 128, device=DEV)
    out = enc(x)
    (out * R).sum().backward()
    torch.cuda.synchronize()
    assert calls, "the 32-true HIP path was not taken"
    params = enc.flat_params()
    p64 = [p.detach().double().cpu().requires_grad_(True) for p in params]
    ref = X.transformer_reference(x.double().cpu(), p64, 2, heads, 0.0, True)
    (ref * R.double().cpu()).sum().backward()
    err = (out.double().cpu() - ref.detach()).abs().max().item() / ref.abs().max().item()
    assert err <= tol, f"forward rel err {err}"
    for i, (p, r) in enumerate(zip(params, p64)):
        e = (p.grad.double().cpu() - r.grad).abs().max().item() / max(r.grad.abs().max().item(), 1e-12)
        assert e <= 10 * tol, f"grad {i} {tuple(p.shape)}: rel err {e}"


def test_transformer_32true_dropout_mask_consistent():
    """32-true transformer with FFN dropout: the dPre1 GEMM regenerates the forward's counter-hash mask from the same
    seed (directional-derivative check of one weight in fp32), and the seeds advance once per forward."""
    from masters_thesis_amd.models.extras import TransformerEncoder

    torch.manual_seed(2)
    enc = TransformerEncoder(3, 128, 2, 4, dropout=0.3).to(DEV)
    enc.precision = "highest"
    enc.train()
    x = torch.randn(32, 40, 3, device=DEV)
    s0 = enc.seeds.clone()
    out = enc(x)
    assert not torch.equal(enc.seeds, s0)
    used = enc.seeds.clone()
    R = torch.randn_like(out)
    (out * R).sum().backward()
    w = enc.blocks[0].fc1.weight
    g = w.grad.clone()
    d = torch.randn_like(w) * 1e-3
    vals = []
    for sgn in (1.0, -1.0):
        with torch.no_grad():
            w.add_(sgn * d)
            enc.seeds.copy_(used)
            enc.seeds.sub_(0x9E3779B97F4A7C15 - (1 << 64))  # the forward advances them again: same mask
            vals.append(float((enc(x) * R).sum()))
            w.sub_(sgn * d)
    fd = (vals[0] - vals[1]) / 2.0
    an = float((g * d).sum())
    assert abs(fd - an) <= 2e-2 * abs(an) + 1e-3, (fd, an)


@pytest.mark.parametrize("prec,tol", [("high", 1e-4), ("highest", 2e-5)])
@pytest.mark.parametrize("norm", ["layernorm", "rmsnorm"])
def test_mlp_32true_hip_path_matches_fp64(prec, tol, norm, monkeypatch):
    """32-true MLP on HIP kernels (ops/extras.py _MlpEncoderF32Fn: csrc/gemm_f32.hip mta_gemm_f32x GEMMs at bf16x3 /
    exact-f32 MFMA, fp32 norms, GELU' fused into the norm backward, ordered bias-gradient column sums) against the
    same encoder in fp64 on the CPU: forward and every parameter gradient.  The HIP path must be the one taken."""
    from masters_thesis_amd.models.extras import MLPEncoder
    from masters_thesis_amd.ops import extras as X

    calls = []
    orig = X._MlpEncoderF32Fn.apply
    monkeypatch.setattr(X._MlpEncoderF32Fn, "apply", lambda *a: calls.append(1) or orig(*a))
    torch.manual_seed(0)
    enc = MLPEncoder(3, 60, 256, 2, 0.0, norm).to(DEV)
    enc.precision = prec
    enc.train()
    x = torch.randn(100, 60, 3, device=DEV)
    R = torch.randn(100, 256, device=DEV)
    out = enc(x)
    (out * R).sum().backward()
    torch.cuda.synchronize()
    assert calls, "the 32-true HIP path was not taken"
    params = enc.flat_params()
    p64 = [p.detach().double().cpu().requires_grad_(True) for p in params]
    ref = X.mlp_reference(x.double().cpu(), p64, 2, norm, 0.0, True)
    (ref * R.double().cpu()).sum().backward()
    err = (out.double().cpu() - ref.detach()).abs().max().item() / ref.abs().max().item()
    assert err <= tol, f"forward rel err {err}"
    for i, (p, r) in enumerate(zip(params, p64)):
        e = (p.grad.double().cpu() - r.grad).abs().max().item() / max(r.grad.abs().max().item(), 1e-12)
        assert e <= 10 * tol, f"grad {i} {tuple(p.shape)}: rel err {e}"


def test_mlp_32true_dropout_masks_consistent():
    """32-true MLP with dropout: the norm backward regenerates the forward's counter-hash mask (a step is
    differentiated exactly: directional derivative check in fp32), and the seeds advance once per forward."""
    from masters_thesis_amd.models.extras import MLPEncoder

    torch.manual_seed(1)
    enc = MLPEncoder(3, 60, 128, 3, 0.3, "layernorm").to(DEV)
    enc.precision = "highest"
    enc.train()
    x = torch.randn(64, 60, 3, device=DEV)
    s0 = enc.seeds.clone()
    out = enc(x)
    assert not torch.equal(enc.seeds, s0)
    used = enc.seeds.clone()
    R = torch.randn_like(out)
    (out * R).sum().backward()
    w = enc.layers[1].weight
    g = w.grad.clone()
    d = torch.randn_like(w) * 1e-3
    vals = []
    for sgn in (1.0, -1.0):
        with torch.no_grad():
            w.add_(sgn * d)
            enc.seeds.copy_(used)
            enc.seeds.sub_(0x9E3779B97F4A7C15 - (1 << 64))  # the forward advances them again: same mask
            vals.append(float((enc(x) * R).sum()))
            w.sub_(sgn * d)
    fd = (vals[0] - vals[1]) / 2.0
    an = float((g * d).sum())
    assert abs(fd - an) <= 2e-2 * abs(an) + 1e-3, (fd, an)


def test_ffn_fragment_major_packing():
    """csrc/tr_ffn.hip frag_pack: the fused FFN's four bf16 fragment-major images (W1, W2, W2^T, W1^T) hold exactly
    the bf16 of the fp32 weights at offset ((n / 16) (K / 32) + k / 32) 512 + ((n % 16) + 16 ((k % 32) / 8)) 8 + k % 8."""
    from masters_thesis_amd.ops._lib import lib

    torch.manual_seed(0)
    w1s = [torch.randn(512, 128, device=DEV) for _ in range(2)]
    w2s = [torch.randn(128, 512, device=DEV) for _ in range(2)]
    out = torch.empty((2, 4, 512, 128), device=DEV, dtype=torch.bfloat16)
    lib().frag_pack([w for l in range(2) for w in (w1s[l], w2s[l], w2s[l], w1s[l])],
                    [out[l, i] for l in range(2) for i in range(4)], [False, False, True, True] * 2)
    for l in range(2):
        for which, src in enumerate((w1s[l], w2s[l], w2s[l].t(), w1s[l].t())):
            N, K = src.shape
            n = torch.arange(N, device=DEV).view(N, 1)
            k = torch.arange(K, device=DEV).view(1, K)
            off = ((n // 16) * (K // 32) + k // 32) * 512 + ((n % 16) + 16 * ((k % 32) // 8)) * 8 + k % 8
            got = out[l, which].reshape(-1)[off.reshape(-1)].view(N, K)
            assert torch.equal(got, src.bfloat16()), (l, which)


@pytest.mark.parametrize("arch", ["mlp", "transformer"])
def test_extras_fused_training_step_matches_autograd(arch):
    """models/extras.py fused_training_step (encoder forward, the one-launch decoder ops.losses.heads_losses_train,
    encoder backward from its dh) against training_step + loss.backward(): same loss, metrics and every gradient."""
    from masters_thesis_amd.models import get_model_class

    g = torch.Generator().manual_seed(0)
    batch = [torch.randn(1, 100, 60, 3, generator=g).to(DEV), (torch.randn(1, 100, 30, 4, generator=g) * 0.01).to(DEV),
             torch.stack([torch.randn(1, generator=g) * 0.01, torch.rand(1, generator=g) * 1e-3 + 1e-4], -1).to(DEV),
             (torch.rand(1, 100, generator=g) * 3 + 1).to(DEV)]
    torch.manual_seed(1)
    kw = dict(hidden_size=128, num_layers=2, dropout=0.0) if arch == "transformer" else dict(hidden_size=256,
                                                                                            num_layers=2, dropout=0.0)
    model = get_model_class("FinancialLstmCombined", arch)(input_size=3, **kw).to(DEV)
    model.train()
    res = []
    for fused in (False, True):
        for p in model.parameters():
            p.grad = torch.zeros_like(p)
        model.train_acc.reset()
        if fused:
            assert model.fused_step_supported(batch)
            loss = model.fused_training_step(batch, 0)
        else:
            loss = model.training_step(batch, 0)
            loss.backward()
        torch.cuda.synchronize()
        res.append((loss.detach().clone(), [p.grad.detach().clone() for p in model.parameters()],
                    model.train_acc.acc.detach().clone()))
    assert _rel(res[0][0], res[1][0]) < 1e-5
    assert _rel(res[0][2], res[1][2]) < 1e-5
    for a, b in zip(res[0][1], res[1][1]):
        assert _rel(a, b) < 1e-4
