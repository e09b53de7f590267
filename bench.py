"""Throughput benchmark: samples/s (whole node) of the flagship training step.

Metric (BASELINE.json): "samples/sec (whole node) synthetic datamodule at 1/2/4/8 MI355X;
p50 step ms".  One sample = one dataset window (100 stocks x 60-day lookback x 3
features, 30-day target).  Config: the reference defaults (`configs/config.yaml`):
``datamodule=synthetic model=small loss=mse trainer=fast`` — LSTM H=64 L=2
(51,074 params), fp32 parameters/activations (trainer precision ``32-true``),
Adam + grad-norm clip 5.0 — random-init weights, synthetic data from the
reference DGP generated on the device.  Every timed step is the full training
step: batch gather, forward, fused loss, backward, gradient all-reduce (N > 1:
the xGMI one-/two-shot kernel of ``parallel/xgmi.py`` inside the step graph; RCCL
when its start-up self-check fails or ``MTA_ALLREDUCE=rccl``, with the reason in
``allreduce_fallback_reason``), clip + Adam, metric accumulation — replayed from
the captured HIP graph exactly as ``train.py`` runs it.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--model M] [--trainer T] [--concurrent k]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

``--gpus N`` without a torchrun environment starts the N ranks itself (parallel/launch.py: ranks 1..N-1 are fresh
child processes re-running this command, this process is rank 0; one rank per GPU, ranks share GPUs only when
fewer are visible).  The record reports the process group's world size, the visible device count and the
gradient all-reduce that ran.

Weak scaling: ``--batch`` windows per GPU per step (global batch = B * N).
Prints exactly one JSON line (rank 0) on stdout.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

# vs_baseline: the same-node reference-equivalent PyTorch path at its best -- ``--backend torch`` (nn.LSTM on MIOpen
# + autograd, heads/loss/optimizer as here) with the whole step captured in a HIP graph, 1 MI355X -- measured by
# this bench, re-measured in round 6 (2026-10-18, profiles/r6_bench_same_node_torch.jsonl: lines 1-5 graph-captured,
# 6-10 ``--no-graphs``; the round-2 figures, profiles/r2_bench_same_node_torch_vs_hip.jsonl, agree to 1-2 %);
# vs_torch_eager divides by the same path run eagerly.  samples/s per GPU keyed (model, loss, per-GPU batch); weak
# scaling: the baseline of N GPUs is N x this.
SAME_NODE_TORCH_GRAPH = {("small", "mse", 1): 515.282, ("medium", "mse", 1): 261.996, ("large", "mse", 1): 132.437,
                         ("small", "mse", 8): 3152.444, ("small", "mse", 64): 4223.826}
SAME_NODE_TORCH_EAGER = {("small", "mse", 1): 168.241, ("medium", "mse", 1): 85.289, ("large", "mse", 1): 42.56,
                         ("small", "mse", 8): 2077.941, ("small", "mse", 64): 4218.843}
# the 8-vCPU CPU replica of the reference step (BASELINE.md yardstick rows); reported as vs_cpu_yardstick
YARDSTICK = {("small", "mse", 1): 59.0, ("small", "nll", 1): 58.0, ("small", "combined", 1): 59.0,
             ("medium", "mse", 1): 21.0, ("large", "mse", 1): 14.0, ("small", "mse", 8): 65.0,
             ("small", "mse", 64): 68.0}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=1,
                    help="windows per GPU per step (reference datamodule default: 1)")
    ap.add_argument("--model", default="small")
    ap.add_argument("--loss", default="mse")
    ap.add_argument("--trainer", default="fast")
    ap.add_argument("--matmul-precision", default="high", choices=["highest", "high", "bf16x3", "medium"])
    ap.add_argument("--backend", default="auto", choices=["auto", "torch"],
                    help="torch = reference-equivalent PyTorch eager path (MIOpen LSTM) for A/B")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--steps-per-graph", type=int, default=None,
                    help="training steps captured per graph (default: the trainer config's steps_per_graph)")
    ap.add_argument("--n-samples", type=int, default=1_000_000, help="synthetic DGP days (reference: 1e6)")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE",
                    help="extra config override (repeatable), e.g. --set model.dropout=0")
    ap.add_argument("--residency", default="device", choices=["device", "stream"],
                    help="device: split resident in HBM; stream: pinned host ring + side-stream H2D per step")
    ap.add_argument("--concurrent", type=int, default=1,
                    help="k independent trainers, one process each, on ONE GPU (the sweep launcher's "
                         "jobs_per_device); value = their summed samples/s over a common start barrier")
    return ap.parse_args(argv)


def _child_barrier() -> None:
    """--concurrent children: wait until every sibling finished its warm-up (file barrier), then time together."""
    d = os.environ.get("MTA_BENCH_BARRIER")
    if not d:
        return
    k, me = int(os.environ["MTA_BENCH_NCHILD"]), int(os.environ["MTA_BENCH_CHILD"])
    Path(d, f"ready.{me}").touch()
    t0 = time.time()
    while len(list(Path(d).glob("ready.*"))) < k:
        if time.time() - t0 > 900:
            raise RuntimeError("concurrent bench: siblings never became ready")
        time.sleep(0.01)


def run_concurrent(args, argv) -> None:
    """Spawn ``args.concurrent`` single-GPU bench processes on the same device and aggregate their lines."""
    import subprocess
    import tempfile

    k = args.concurrent
    if not 1 < k <= 8:
        raise SystemExit("--concurrent: 2..8 processes per GPU")
    raw = list(sys.argv[1:] if argv is None else argv)
    child_argv, skip = [], False
    for a in raw:
        if skip:
            skip = False
            continue
        if a == "--concurrent":
            skip = True
            continue
        if a.startswith("--concurrent="):
            continue
        child_argv.append(a)
    with tempfile.TemporaryDirectory(prefix="mta_bench_") as d:
        procs = []
        for i in range(k):
            env = dict(os.environ, MTA_BENCH_BARRIER=d, MTA_BENCH_NCHILD=str(k), MTA_BENCH_CHILD=str(i))
            # trainers time-slicing one GPU: the pipelined LSTM's cross-workgroup waits may sit out another
            # process's slice, so they poll 16x longer before giving up (a give-up still fails the run)
            env.setdefault("MTA_LSTM_SPIN_LIMIT", str(1 << 25))
            env.setdefault("MTA_ADAM_SPIN_LIMIT", str(1 << 26))
            env.setdefault("GPU_MAX_HW_QUEUES", "1")  # one hardware queue per trainer: k queues, no oversubscription
            for v in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
                env.pop(v, None)
            procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve()), *child_argv], env=env,
                                          stdout=subprocess.PIPE, text=True))
        outs = [p.communicate()[0] for p in procs]
        rcs = [p.returncode for p in procs]
    if any(rcs):
        raise SystemExit(f"concurrent bench: child exit codes {rcs}")
    recs = [json.loads([ln for ln in o.splitlines() if ln.startswith("{")][-1]) for o in outs]
    rec = dict(recs[0])
    total = sum(r["value"] for r in recs)
    rec["value"] = round(total, 3)
    rec["ms_per_step"] = round(max(r["ms_per_step"] for r in recs), 4)
    rec["p50_step_ms"] = round(max(r["p50_step_ms"] for r in recs), 4)
    rec["p90_step_ms"] = round(max(r["p90_step_ms"] for r in recs), 4)
    rec["concurrent_trainers"] = k
    rec["per_trainer_samples_per_s"] = [r["value"] for r in recs]
    rec["vs_baseline"] = None if recs[0]["vs_baseline"] is None else round(
        total / (recs[0]["value"] / recs[0]["vs_baseline"]), 3)
    rec["vs_torch_eager"] = None
    rec["vs_cpu_yardstick"] = None
    rec["config"] = dict(rec["config"], parallelism=f"{k} independent trainers on 1 GPU (trial packing)",
                         global_batch=rec["config"]["global_batch"] * k)
    print(json.dumps(rec), flush=True)


def main(argv=None):
    args = parse_args(argv)
    if args.concurrent > 1 and not os.environ.get("MTA_BENCH_CHILD"):
        run_concurrent(args, argv)
        return
    from masters_thesis_amd.config import compose
    from masters_thesis_amd.data import FinancialLstmDataModule
    from masters_thesis_amd.engine import Trainer
    from masters_thesis_amd.models import get_model_class, model_params_from_config
    from masters_thesis_amd.parallel import dist as pdist
    from masters_thesis_amd.parallel import launch

    if args.gpus > 1 and not launch.in_launched_job():
        launch.launch_script_ranks(args.gpus)  # before anything touches the GPU
    denv = pdist.init_distributed()
    world = denv.world_size
    pg_world = torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1
    if not (world == pg_world == args.gpus):
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the job has WORLD_SIZE={world} (process group "
                         f"{pg_world}): refusing to report a different world than asked for")
    dev = denv.device
    torch.manual_seed(1234 + denv.rank)

    cfg, _, _ = compose(REPO / "configs", "config", [
        f"model={args.model}", f"loss={args.loss}", f"trainer={args.trainer}",
        f"datamodule.batch_size={args.batch}", f"datamodule.n_samples={args.n_samples}",
        f"datamodule.residency={args.residency}", *args.set])
    if args.backend == "torch":
        cfg.model["backend"] = "torch"
    t_data = time.perf_counter()
    dm = FinancialLstmDataModule.from_config(cfg.datamodule, cache=False, device=dev, rank=denv.rank,
                                             world_size=world)
    dm.setup("fit")
    log(f"[bench] rank {denv.rank}: {dm.n_windows} windows built on {dev} in {time.perf_counter() - t_data:.1f}s")

    ModelClass = get_model_class(cfg.loss.module_class, cfg.model.get("arch", "lstm"))
    model = ModelClass(**model_params_from_config(cfg))
    if args.backend == "torch":
        model.allow_torch_capture = not args.no_graphs  # eager warm-up first: measured capture-safe here
    trainer = Trainer(max_epochs=1, gradient_clip_val=cfg.trainer.gradient_clip_val, precision=cfg.trainer.precision,
                      enable_progress_bar=False, enable_model_summary=False, logger=None, callbacks=[],
                      use_hip_graphs=not args.no_graphs, matmul_precision=args.matmul_precision,
                      **({"steps_per_graph": args.steps_per_graph} if args.steps_per_graph is not None else
                         {"steps_per_graph": cfg.trainer.steps_per_graph} if "steps_per_graph" in cfg.trainer
                         else {}))
    trainer._setup_env()
    trainer._setup_model(model)
    trainer._configure_optimizers(model)
    model.train()

    loader = dm.train_dataloader()
    step = trainer.make_train_stepper(loader)  # full batches; epoch roll-over reshuffles like fit()
    S = max(1, trainer.steps_per_graph if trainer._can_group(loader) else 1)
    # warmup: eager runs + capture of the single-step and grouped graphs, then W steps of replays
    for _ in range(max(args.warmup, 0)):
        step()
    for _ in range(trainer.graph_warmup_steps + 2 if S > 1 else 0):
        step(S)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    _child_barrier()
    pdist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    evs = []
    t0 = time.perf_counter()
    done = 0
    while done < args.steps:
        n = S if args.steps - done >= S else 1
        if dev.type == "cuda":
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        step(n)
        if dev.type == "cuda":
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            evs.extend([(e0, e1, n)] * n)
        done += n
    host_issue_s = time.perf_counter() - t0  # host time to issue the K steps (launch-bound when ~ elapsed)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    pdist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    elapsed = pdist.all_reduce_max(elapsed, dev)
    # gradient all-reduce alone (world > 1): mean over 50 back-to-back syncs of the flat bucket, after the
    # timed region (the timed steps include it)
    allreduce_us = None
    if world > 1 and dev.type == "cuda":
        for _ in range(5):
            trainer.ddp.allreduce_grads()
        torch.cuda.synchronize()
        a0 = time.perf_counter()
        for _ in range(50):
            trainer.ddp.allreduce_grads()
        torch.cuda.synchronize()
        allreduce_us = pdist.all_reduce_max((time.perf_counter() - a0) / 50 * 1e6, dev)
    step_ms = sorted(a.elapsed_time(b) / n for a, b, n in evs) if evs else [elapsed * 1e3 / args.steps]
    p50 = pdist.all_reduce_max(step_ms[len(step_ms) // 2], dev)
    p90 = pdist.all_reduce_max(step_ms[min(len(step_ms) - 1, (len(step_ms) * 9) // 10)], dev)
    ms_per_step = elapsed * 1e3 / args.steps
    value = args.batch * world * args.steps / elapsed
    nonfinite = float(trainer.optimizer.nonfinite.item())
    trainer._check_device_health()  # raises if a pipelined hand-off gave up (garbage steps)
    key = (args.model, args.loss, args.batch)
    eff_prec = trainer._effective_matmul_precision()
    if denv.rank == 0:
        log(f"[bench] p50 step {p50:.3f} ms, mean {ms_per_step:.3f} ms, graphs={'on' if trainer._graphs else 'off'}, "
            f"nonfinite={nonfinite}, static_batches={trainer._static_ok(loader)}")
        rec = {
            "metric": "samples/sec (whole node) synthetic datamodule; p50 step ms",
            "value": round(value, 3),
            "unit": "samples/s",
            "n_gpus": world,
            "world_size": pg_world,
            "visible_devices": torch.cuda.device_count() if dev.type == "cuda" else 0,
            "process_group": denv.backend or "none",
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "p50_step_ms": round(p50, 4),
            "p90_step_ms": round(p90, 4),
            "host_issue_ms_per_step": round(host_issue_s * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(value / (world * SAME_NODE_TORCH_GRAPH[key]), 3)
                            if key in SAME_NODE_TORCH_GRAPH and args.backend == "auto" else None),
            "baseline": "same-node PyTorch-ROCm reference path (MIOpen nn.LSTM + autograd, step captured in a HIP "
                        "graph), x n_gpus",
            "vs_torch_eager": (round(value / (world * SAME_NODE_TORCH_EAGER[key]), 3)
                               if key in SAME_NODE_TORCH_EAGER and args.backend == "auto" else None),
            "vs_cpu_yardstick": (round(value / YARDSTICK[key], 3) if key in YARDSTICK else None),
            "allreduce": trainer.ddp.backend_name,
            "allreduce_fallback_reason": trainer.ddp.fallback_reason,
            "allreduce_us": round(allreduce_us, 2) if allreduce_us is not None else None,
            "grad_bucket_bytes": int(trainer.flat.padded * 4),
            # the compute dtype that actually ran: the extras' bf16 HIP kernels run only at matmul precision
            # "medium" (bf16-mixed); under 32-true they run the fp32 graph.  The LSTM keeps fp32 parameters and
            # activations; its recurrent matmuls run at matmul_precision (bf16x3 MFMA for "high")
            "dtype": "bf16" if eff_prec == "medium" else "fp32",
            "matmul_dtype": {"medium": "bf16",
                             "high": ("LSTM fwd fp16x2 (TF32-class: fp16 activations, fp16 hi+lo weights), bwd bf16x3"
                                      if cfg.model.get("arch", "lstm") == "lstm" else "bf16x3"),
                             "bf16x3": "bf16x3 (fp32-accurate)", "highest": "fp32"}[eff_prec],
            "data": "synthetic (reference DGP, generated on device), random-init weights",
            "config": {
                "model": f"{type(model).__name__} model={args.model} "
                         f"({cfg.model.get('arch', 'lstm')} H={cfg.model.hidden_size} L={cfg.model.num_layers}, "
                         f"{sum(p.numel() for p in model.parameters())} params)",
                "global_batch": args.batch * world,
                "seq_len": int(cfg.datamodule.lookback_window),
                "parallelism": f"dp{world}",
                "per_gpu_batch_windows": args.batch,
                "sequences_per_window": 100,
                "trainer": args.trainer,
                "precision": cfg.trainer.precision,
                "matmul_precision": eff_prec,
                "backend": "hip" if args.backend == "auto" else "torch-miopen",
                "hip_graphs": not args.no_graphs,
                "steps_per_graph": S,
                "residency": args.residency,
                # optional fused paths in force (env switches, ops/extras.py / ops/optim.py)
                "fused_paths": _fused_paths(cfg, trainer),
            },
        }
        print(json.dumps(rec), flush=True)
    pdist.destroy()


def _fused_paths(cfg, trainer) -> dict:
    arch = cfg.model.get("arch", "lstm")
    if arch == "transformer":
        from masters_thesis_amd.ops import extras as X

        return {"transformer_ffn": bool(X._TR_FFN[0]), "transformer_attn": bool(X._TR_ATTN[0]),
                "transformer_wgrad_nn": bool(X._TR_FFN[0] and X._TR_WGRAD_NN[0])}
    if arch == "mlp":
        # producers on (single process, or world > 1 with the xGMI all-reduce's clip-norm partials)
        return {"optimizer_grad_producers": bool(getattr(trainer, "grad_producers", False))
                and os.environ.get("MTA_OPTIM_PRODUCERS", "1") != "0",
                "clip_norm_from_allreduce": trainer.ddp.norm_parts is not None}
    return {}


if __name__ == "__main__":
    main()
