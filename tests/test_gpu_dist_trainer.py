"""Multi-rank TRAINER steps on one MI355X (ranks share cuda:0; gloo process group for the host collectives).

The reference's DDP is Lightning's implicit one (`/root/reference/train.py:169-180`); here every rank runs the real
``Trainer`` stepper (``make_train_stepper``: eager warm-up steps, then the whole step captured in a HIP graph and
replayed), so these tests cover what the driver's 8-GPU SCALE run executes, minus the xGMI link itself:

* ``xgmi``: ``MTA_ALLREDUCE=xgmi`` -- the gradient sync is the xGMI all-reduce kernel INSIDE the captured step,
  with the backward-overlapped ranges (``FlatDDP.begin_backward`` -> ``grad_ready`` from the encoder backward ->
  side-stream launches -> join -> fused clip + AdamW).  Replicas must stay bit-identical, and the parameters after
  the steps must match ONE rank running the global batch (world x B windows per step: the same windows, since
  rank r takes positions r, r + world, ... of the epoch order).
* ``gloo``: the host-staged gloo sync after the replayed fwd/bwd graph (the r3 rehearsal path).  4 ranks of the
  graphed bf16 transformer went non-finite from the second replay on (profiles/r3_s3_dist_rehearsal.txt); the
  root cause was a captured hipMemsetAsync node (profiles/r4_nan_root_cause.txt).  Regression: ~35 graphed steps,
  every gradient norm finite.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, model, batch, steps, sync, q, extra_env, trainer="gpu_fast", spg=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world), MTA_DIST_BACKEND="gloo")
    if sync == "xgmi":
        os.environ["MTA_ALLREDUCE"] = "xgmi"
    else:
        os.environ["MTA_ALLREDUCE"] = "rccl"  # no xGMI: the process group's (gloo) all-reduce after the graph
    os.environ.update(extra_env)
    try:
        import sys

        sys.path.insert(0, REPO)
        from masters_thesis_amd.config import compose
        from masters_thesis_amd.data import FinancialLstmDataModule
        from masters_thesis_amd.engine import Trainer
        from masters_thesis_amd.models import get_model_class, model_params_from_config
        from masters_thesis_amd.parallel import dist as pdist

        denv = pdist.init_distributed()
        dev = denv.device
        torch.manual_seed(0)
        cfg, _, _ = compose(os.path.join(REPO, "configs"), "config", [
            f"model={model}", "loss=mse", f"trainer={trainer}", f"datamodule.batch_size={batch}",
            "datamodule.n_samples=20000", "model.dropout=0"])
        dm = FinancialLstmDataModule.from_config(cfg.datamodule, cache=False, device=dev, rank=denv.rank,
                                                 world_size=denv.world_size)
        dm.setup("fit")
        mcls = get_model_class(cfg.loss.module_class, cfg.model.get("arch", "lstm"))
        net = mcls(**model_params_from_config(cfg))
        tr = Trainer(max_epochs=1, gradient_clip_val=cfg.trainer.gradient_clip_val, precision=cfg.trainer.precision,
                     enable_progress_bar=False, enable_model_summary=False, logger=None, callbacks=[],
                     use_hip_graphs=True, steps_per_graph=spg)
        tr.keep_graphs = True  # graph_census() below: node types of every captured step graph
        tr._setup_env()
        tr._setup_model(net)
        tr._configure_optimizers(net)
        net.train()
        info = {"backend": tr.ddp.backend_name, "in_graph": tr._allreduce_in_graph(),
                "overlap": bool(getattr(tr.ddp, "overlap", False)),
                "producers": bool(getattr(tr, "grad_producers", False)),
                "norm_from_allreduce": tr.ddp.norm_parts is not None}
        # the gradient the optimizer sees at step 1 (summed over ranks, times the 1/world it applies) and the clip
        # norm it computes from it: the first step is an eager warm-up step, so the wrapper sees it
        snap = {}
        opt_step = tr.optimizer.step

        def step_and_snapshot(max_norm=0.0, grad_scale=1.0, zero_grad=False, **kw):
            first = "grad" not in snap
            if first:
                torch.cuda.synchronize()
                snap["grad"] = (tr.flat.grad.detach().double() * grad_scale).cpu().numpy().copy()
            opt_step(max_norm, grad_scale, zero_grad, **kw)
            if first:
                snap["norm"] = float(tr.optimizer.grad_norm.item())

        tr.optimizer.step = step_and_snapshot
        loader = dm.train_dataloader()
        step = tr.make_train_stepper(loader)
        launches = []
        info["grouped"] = tr._can_group(loader)
        done = 0
        while done < steps:
            n = spg if (spg > 1 and steps - done >= spg) else 1
            step(n)
            done += n
            launches.append(tr.ddp._launches if world > 1 else 0)
        torch.cuda.synchronize()
        tr._check_device_health()
        info["nonfinite"] = float(tr.optimizer.nonfinite.item())
        info["launches"] = launches
        info["graphed"] = bool(tr._graphs)
        info["grad1"], info["norm1"] = snap.get("grad"), snap.get("norm")
        info["census"] = [(str(k), c) for k, c in tr.graph_census().items()] if tr._graphs else []
        # numpy (pickled by value): a torch CPU tensor would travel as a shared-memory fd the exiting worker closes
        q.put((rank, tr.flat.data.detach().cpu().numpy().copy(), info, None))
        pdist.barrier()
        if tr.ddp.xgmi is not None:
            tr.ddp.xgmi.close()
        pdist.destroy()
    except Exception:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, None, None, traceback.format_exc()))


def _run(world, model, batch, steps, sync, extra_env=None, timeout=280, trainer="gpu_fast", spg=1):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, model, batch, steps, sync, q, extra_env or {}, trainer,
                                               spg))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=timeout) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for rank, _, _, err in res:
        assert err is None, f"rank {rank}:\n{err}"
    return [(rank, torch.from_numpy(p), info, err) for rank, p, info, err in res]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("model,trainer,tol", [("small", "fast", 1e-5), ("mlp_small", "gpu_fast", 2e-3),
                                               ("transformer_encoder", "gpu_fast", 2e-3),
                                               ("mlp_large", "gpu_fast", 2e-3)])
def test_step1_summed_gradient_matches_global_batch(model, trainer, tol):
    """The all-reduce checked where it can be checked sharply: the gradient the optimizer receives at step 1 (sum over
    2 ranks x B=1 through the xGMI kernel, times 1/world) against ONE rank on the same 2 windows (B=2), and the clip
    norm computed from it -- before Adam, which turns near-zero gradients' rounding noise into lr-sized steps.

    Tolerances: fp32 LSTM (32-true) 1e-5 relative (norm of the difference over the norm of the gradient; the two runs
    differ only in the order the kernels sum per-sequence weight-gradient contributions and the loss mean over two
    windows); bf16 extras 2e-3 (bf16 GEMM tiles of a 100- vs 200-row batch round their inputs identically but split
    K differently: fp32 partial sums in another order, relative to bf16-rounded products)."""
    dist_res = _run(2, model, 1, 1, "xgmi", trainer=trainer)
    (_, _, i0, _), (_, _, i1, _) = dist_res
    assert i0["backend"] == "xgmi", i0["backend"]
    ((_, _, iref, _),) = _run(1, model, 2, 1, "none", trainer=trainer)
    g0, g1, gref = (torch.from_numpy(i["grad1"]) for i in (i0, i1, iref))
    assert torch.equal(g0, g1), "ranks received different summed gradients"
    rel = ((g0 - gref).norm() / gref.norm()).item()
    nrel = abs(i0["norm1"] - iref["norm1"]) / iref["norm1"]
    print(f"[{model}] step-1 gradient 2 ranks x B=1 vs 1 rank x B=2: rel {rel:.3g}, clip-norm rel {nrel:.3g}")
    assert gref.norm().item() > 0
    assert rel <= tol, rel
    assert nrel <= tol, (i0["norm1"], iref["norm1"])
    # the clip norm comes from the all-reduce kernel's partials of the reduced gradient (world 2) and the gradient
    # producers stay on (mlp_large's big weight gradients overwrite their ranges) -- VERDICT r5 next-round #5
    assert i0["norm_from_allreduce"] and i0["producers"], i0
    assert iref["producers"], iref


@pytest.mark.timeout(600)
@pytest.mark.parametrize("model", ["mlp_small", "transformer_encoder"])
def test_trainer_xgmi_in_graph_two_ranks(model):
    steps = 6
    # overlap threshold lowered so mlp_small's layer ranges are reduced on the side stream during the backward too
    env = {"MTA_DDP_OVERLAP_MIN_KB": "16"}
    dist_res = _run(2, model, 1, steps, "xgmi", env)
    (_, p0, info0, _), (_, p1, info1, _) = dist_res
    assert info0["backend"] == "xgmi" and info0["in_graph"] and info0["overlap"], info0
    assert info0["graphed"], info0
    _assert_kernel_only(info0["census"])
    # the backward reported ranges during the backward (side-stream launches) besides the final sync
    assert min(info0["launches"]) >= 2, info0
    assert info0["nonfinite"] == 0 and info1["nonfinite"] == 0
    assert torch.isfinite(p0).all()
    assert torch.equal(p0, p1), "replicas diverged"
    ((_, pref, info_ref, _),) = _run(1, model, 2, steps, "none")
    assert info_ref["nonfinite"] == 0
    # 6 AdamW steps at lr 1e-4 move a parameter by <= ~6 x lr.  Per-rank vs global-batch bf16 GEMMs differ in tile
    # order (fp32 accumulation, last-bit differences), and Adam normalises every gradient element: an element whose
    # gradient is ~0 can take a different sign and move by up to lr per step.  So: every element within the Adam
    # step bound, and all but a small fraction of them within 2e-5 (rtol 1e-4 of typical weights)
    diff = (p0 - pref).abs()
    moved = (pref - _run_init(model)).abs().max().item()
    frac = (diff > 2e-5 + 1e-4 * pref.abs()).float().mean().item()
    stats = f"max {diff.max().item():.3g}, mean {diff.mean().item():.3g}, frac>tol {frac:.4g}, moved {moved:.3g}"
    print(f"[{model}] 2 ranks x B=1 vs 1 rank x B=2 after {steps} steps: {stats}")
    assert moved > 1e-4, "parameters did not move: " + stats
    assert diff.max().item() <= 1.5 * steps * 1e-4, stats
    assert frac < 0.02, stats


def _assert_kernel_only(census):
    """The world-2 step graphs (xGMI all-reduce inside) hold kernel nodes only (tests/test_gpu_graphs.py)."""
    assert census, "no graph captured"
    for key, c in census:
        print(f"census {key}: {c}")
        assert c["kernel"] > 0 and c["memset"] == 0 and c["memcpy"] == 0 and c["other"] == 0, (key, c)


_INIT = {}


def _run_init(model):
    """Initial flat parameters (seed 0, as the workers)."""
    if model not in _INIT:
        import sys

        sys.path.insert(0, REPO)
        from masters_thesis_amd.config import compose
        from masters_thesis_amd.models import get_model_class, model_params_from_config
        from masters_thesis_amd.ops.optim import FlatParameters

        torch.manual_seed(0)
        cfg, _, _ = compose(os.path.join(REPO, "configs"), "config",
                            [f"model={model}", "loss=mse", "trainer=gpu_fast", "model.dropout=0"])
        net = get_model_class(cfg.loss.module_class, cfg.model.get("arch", "lstm"))(**model_params_from_config(cfg))
        _INIT[model] = FlatParameters(net.parameters(), device=torch.device("cpu")).data.clone()
    return _INIT[model]


@pytest.mark.timeout(600)
def test_trainer_gloo_four_ranks_graphed_transformer_stays_finite():
    """Regression of the r3 open finding: 4 ranks, graphed bf16 transformer, host-staged gloo sync."""
    res = _run(4, "transformer_encoder", 1, 35, "gloo")
    ps = [r[1] for r in res]
    for rank, p, info, _ in res:
        assert info["graphed"] and not info["in_graph"], info
        assert info["nonfinite"] == 0, (rank, info)
        assert torch.isfinite(p).all(), rank
    for p in ps[1:]:
        assert torch.equal(ps[0], p), "replicas diverged"


@pytest.mark.timeout(600)
def test_trainer_xgmi_four_ranks_two_shot_transformer():
    """4 ranks: the transformer's 3.2 MB gradient takes the two-shot path (> 512 KB, world > 2) with uneven chunks;
    overlapped layer ranges on the side stream; 20 graphed steps, replicas bit-identical and finite."""
    res = _run(4, "transformer_encoder", 1, 20, "xgmi")
    ps = [r[1] for r in res]
    for rank, p, info, _ in res:
        assert info["backend"] == "xgmi" and info["in_graph"] and info["overlap"], info
        assert info["nonfinite"] == 0, (rank, info)
        assert torch.isfinite(p).all(), rank
    for p in ps[1:]:
        assert torch.equal(ps[0], p), "replicas diverged"


@pytest.mark.timeout(600)
def test_trainer_xgmi_grouped_lstm_two_ranks():
    """The headline model under the driver's multi-GPU configuration: LSTM small, 32-true, xGMI all-reduce inside
    GROUPED step graphs (4 training steps per captured graph, each with its own all-reduce on the device-resident
    channel epochs).  Replicas bit-identical; parameters vs one rank on the global batch."""
    steps = 12
    res = _run(2, "small", 1, steps, "xgmi", trainer="fast", spg=4)
    (_, p0, info0, _), (_, p1, info1, _) = res
    assert info0["backend"] == "xgmi" and info0["in_graph"] and info0["grouped"], info0
    _assert_kernel_only(info0["census"])
    assert info0["nonfinite"] == 0 and info1["nonfinite"] == 0
    assert torch.isfinite(p0).all()
    assert torch.equal(p0, p1), "replicas diverged"
    ((_, pref, info_ref, _),) = _run(1, "small", 2, steps, "none", trainer="fast", spg=4)
    diff = (p0 - pref).abs()
    frac = (diff > 2e-5 + 1e-4 * pref.abs()).float().mean().item()
    stats = f"max {diff.max().item():.3g}, mean {diff.mean().item():.3g}, frac>tol {frac:.4g}"
    print(f"[small LSTM] 2 ranks x B=1 vs 1 rank x B=2 after {steps} grouped steps: {stats}")
    assert diff.max().item() <= 1.5 * steps * 1e-4, stats
    assert frac < 0.02, stats
