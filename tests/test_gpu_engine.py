"""Engine-level GPU tests: streaming (pinned ring + side-stream H2D) vs HBM-resident batches."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _data(W=23):
    g = torch.Generator().manual_seed(0)
    return [torch.randn(W, 100, 60, 3, generator=g), torch.randn(W, 100, 30, 4, generator=g),
            torch.stack([torch.randn(W, generator=g) * 0.1, torch.rand(W, generator=g) + 0.2], -1),
            torch.rand(W, 100, generator=g) * 3 + 1]


def test_streaming_loader_static_batches_match_device_gather():
    from masters_thesis_amd.data.datamodule import TensorBatchLoader
    from masters_thesis_amd.data.prefetch import StreamingLoader

    data = _data()
    host = [t.pin_memory() for t in data]
    ld = StreamingLoader(TensorBatchLoader(host, 2, shuffle=True, seed=4), DEV, slots=3, threads=2)
    assert ld.supports_static()
    for epoch in range(2):
        nfull = ld.begin_epoch(epoch)
        idx = ld._epoch_idx
        for s in range(nfull):
            ld.before_static_step()
            bufs = ld.gather_static()
            ld.after_static_step()
            rows = idx[s * 2:(s + 1) * 2]
            for b, t in zip(bufs, data):
                torch.testing.assert_close(b.cpu(), t[rows], rtol=0, atol=0)
        tail = ld.tail_batch()
        assert tail is not None and tail[0].shape[0] == 1
    assert ld.bytes_copied > 0
    ld.close()


def test_trainer_streaming_equals_resident():
    from masters_thesis_amd.data.datamodule import TensorBatchLoader
    from masters_thesis_amd.data.prefetch import StreamingLoader
    from masters_thesis_amd.engine import Trainer
    from masters_thesis_amd.models import FinancialLstmMse

    def run(stream):
        torch.manual_seed(3)
        model = FinancialLstmMse(dropout=0.0)
        data = _data(17)
        if stream:
            ld = StreamingLoader(TensorBatchLoader([t.pin_memory() for t in data], 1, shuffle=True, seed=0), DEV)
        else:
            ld = TensorBatchLoader([t.to(DEV) for t in data], 1, shuffle=True, seed=0)
        tr = Trainer(gradient_clip_val=5.0, enable_progress_bar=False, enable_model_summary=False,
                     use_hip_graphs=True, matmul_precision="highest")
        tr._setup_env()
        tr._setup_model(model)
        tr._configure_optimizers(model)
        model.train()
        step = tr.make_train_stepper(ld)
        for _ in range(40):  # crosses two epoch boundaries (17 batches per epoch)
            step()
        torch.cuda.synchronize()
        return tr.flat.data.clone()

    # float atomics in the weight-gradient kernel make runs differ in the last bits
    torch.testing.assert_close(run(True), run(False), rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("cls_name", ["FinancialLstmMse", "FinancialLstmNll", "FinancialLstmCombined"])
@pytest.mark.parametrize("B,H,L", [(1, 64, 2), (2, 64, 2), (1, 16, 2), (1, 16, 1), (2, 32, 1)])
def test_fused_training_step_matches_autograd(cls_name, B, H, L):
    """models/lstm.py fused_training_step (pipelined fwd + one-launch decoder + pipelined bwd, no autograd)
    against training_step + loss.backward(): same loss, gradients and epoch-metric sums, dropout on."""
    import masters_thesis_amd.models as M
    from masters_thesis_amd.ops.optim import FlatParameters

    data = [t[:B].to(DEV) for t in _data(4)]
    out = []
    for fused in (False, True):
        torch.manual_seed(11)
        model = getattr(M, cls_name)(hidden_size=H, num_layers=L, dropout=0.2).to(DEV)
        model.lstm.seeds.copy_(torch.arange(8, device=DEV) * 977 + 5)
        model.matmul_precision = "highest"
        flat = FlatParameters(model.parameters())
        model.train()
        assert model.fused_step_supported(data)
        if fused:
            loss = model.fused_training_step(data, 0)
        else:
            loss = model.training_step(data, 0)
            loss.backward()
        torch.cuda.synchronize()
        out.append((float(loss), flat.grad.clone(), model.train_acc.acc.clone(), model.lstm.seeds.clone()))
    (la, ga, aa, sa), (lb, gb, ab, sb) = out
    assert abs(la - lb) <= 1e-5 * abs(la), (la, lb)
    torch.testing.assert_close(gb, ga, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(ab, aa, rtol=1e-6, atol=0)
    assert torch.equal(sa, sb)  # dropout seeds advanced once by both paths


def test_deterministic_mode_runs_are_bit_identical():
    """Trainer(deterministic=True): ordered per-chunk weight-gradient reductions (csrc/lstm_wgrad.h
    wgrad_reduce_kernel) instead of f32 atomics -> two training runs give bit-identical parameters; the
    result matches the atomic (default) path to rounding."""
    from masters_thesis_amd.data.datamodule import TensorBatchLoader
    from masters_thesis_amd.engine import Trainer
    from masters_thesis_amd.models import FinancialLstmCombined
    from masters_thesis_amd.ops import lstm as op

    def run(det):
        torch.manual_seed(3)
        model = FinancialLstmCombined(dropout=0.2)
        ld = TensorBatchLoader([t.to(DEV) for t in _data(9)], 1, shuffle=True, seed=0)
        tr = Trainer(gradient_clip_val=5.0, enable_progress_bar=False, enable_model_summary=False,
                     use_hip_graphs=True, matmul_precision="high", deterministic=det)
        tr._setup_env()
        tr._setup_model(model)
        tr._configure_optimizers(model)
        model.lstm.seeds.copy_(torch.arange(8, device=DEV) + 17)
        model.train()
        step = tr.make_train_stepper(ld)
        for _ in range(20):
            step()
        torch.cuda.synchronize()
        op.set_deterministic(False)
        return tr.flat.data.clone()

    a, b = run(True), run(True)
    assert torch.equal(a, b)
    torch.testing.assert_close(run(False), a, rtol=1e-4, atol=1e-6)


def test_grouped_step_graphs_match_single_steps():
    """Trainer(steps_per_graph=S): S consecutive steps captured as one graph (one launch per group, each step
    gathering its own batch through the device cursor) train exactly like S single-step replays —
    bit-identical parameters in deterministic mode, across epoch roll-overs (9 batches per epoch)."""
    from masters_thesis_amd.data.datamodule import TensorBatchLoader
    from masters_thesis_amd.engine import Trainer
    from masters_thesis_amd.models import FinancialLstmCombined
    from masters_thesis_amd.ops import lstm as op

    def run(S):
        torch.manual_seed(3)
        model = FinancialLstmCombined(dropout=0.2)
        ld = TensorBatchLoader([t.to(DEV) for t in _data(9)], 1, shuffle=True, seed=0)
        tr = Trainer(gradient_clip_val=5.0, enable_progress_bar=False, enable_model_summary=False,
                     use_hip_graphs=True, matmul_precision="high", deterministic=True, steps_per_graph=S)
        tr._setup_env()
        tr._setup_model(model)
        tr._configure_optimizers(model)
        model.lstm.seeds.copy_(torch.arange(8, device=DEV) + 17)
        model.train()
        assert tr._can_group(ld) == (S > 1)
        step = tr.make_train_stepper(ld)
        for _ in range(24 // S):
            step(S)
        torch.cuda.synchronize()
        op.set_deterministic(False)
        acc = model.train_acc.acc.clone() if hasattr(model, "train_acc") else None
        return tr.flat.data.clone(), acc, model.lstm.seeds.clone()

    (pa, aa, sa), (pb, ab, sb) = run(1), run(4)
    assert torch.equal(pa, pb)
    assert torch.equal(sa, sb)
    if aa is not None:
        assert torch.equal(aa, ab)


@pytest.mark.parametrize("B,L,dropout", [(1, 2, 0.2), (3, 1, 0.0), (2, 3, 0.2)])
def test_deferred_gather_equals_gather_kernel(B, L, dropout, monkeypatch):
    """The batch gather folded into the pipelined forward launch (layer 0 reads x through the permutation,
    the static buffers are filled in-launch, the cursor advances once per launch) trains bit-identically to
    the separate gather kernel, across an epoch roll-over and with grouped step graphs."""
    from masters_thesis_amd.data.datamodule import TensorBatchLoader
    from masters_thesis_amd.engine import Trainer
    from masters_thesis_amd.models import FinancialLstmCombined

    def run(defer):
        monkeypatch.setenv("MTA_DEFER_GATHER", "1" if defer else "0")
        torch.manual_seed(3)
        model = FinancialLstmCombined(num_layers=L, dropout=dropout)
        ld = TensorBatchLoader([t.to(DEV) for t in _data(19)], B, shuffle=True, seed=1)
        tr = Trainer(gradient_clip_val=5.0, enable_progress_bar=False, enable_model_summary=False,
                     use_hip_graphs=True, matmul_precision="high", steps_per_graph=4, deterministic=True)
        tr._setup_env()
        tr._setup_model(model)
        tr._configure_optimizers(model)
        model.train()
        step = tr.make_train_stepper(ld)
        launched = []
        orig = ld.gather_static

        def spy(defer=False):
            launched.append(defer)
            return orig(defer=defer)

        ld.gather_static = spy
        for _ in range(30):
            step()
        step(4)
        torch.cuda.synchronize()
        tr._check_device_health()
        return [p.detach().clone() for p in model.parameters()], launched, [b.clone() for b in ld._static]

    from masters_thesis_amd.ops import extras as extras_op
    from masters_thesis_amd.ops import lstm as lstm_op

    try:  # deterministic weight-gradient reductions: the two runs must agree bit for bit
        p_def, l_def, s_def = run(True)
        p_ref, l_ref, s_ref = run(False)
    finally:
        lstm_op.set_deterministic(False)
        if hasattr(extras_op, "set_deterministic"):
            extras_op.set_deterministic(False)
    assert l_def and all(l_def) and not any(l_ref)
    for a, b in zip(s_def, s_ref):  # the static buffers hold the same last batch
        torch.testing.assert_close(a, b, rtol=0, atol=0)
    for a, b in zip(p_def, p_ref):
        torch.testing.assert_close(a, b, rtol=0, atol=0)
