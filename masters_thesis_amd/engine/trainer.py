"""Training engine: fit / validate / test loops with Lightning-equivalent semantics.

Reference behaviour (Lightning ``Trainer`` as configured in `train.py:169-198`):
sanity validation (2 batches), per-epoch training with ``gradient_clip_val`` norm
clipping, validation every ``check_val_every_n_epoch``, ``ModelCheckpoint`` and
``LearningRateMonitor`` callbacks, ``ReduceLROnPlateau`` stepped at the validation
frequency on ``loss/total/val`` (`src/model.py:156-172`), epoch-level logging of
``self.log(..., on_epoch=True)`` values, ``trainer.test`` on the current weights.

MI355X execution model:

* one process per GPU (``parallel.dist``), gradients in one flat buffer,
  one RCCL all-reduce per step (``parallel.ddp.FlatDDP``), metrics synced with
  one fused all-reduce per epoch (fixes the rank-local monitor of SURVEY Q2);
* the optimizer is the fused clip+Adam HIP kernel pair (``ops.optim.FusedAdam``),
  swapped in for ``torch.optim.Adam/AdamW`` returned by ``configure_optimizers``;
* with an HBM-resident dataset the batch is assembled on the device by one gather
  kernel (indices from a per-epoch device permutation + device cursor), so after
  ``graph_warmup_steps`` eager steps the WHOLE train step — gather, forward, fused
  heads/losses/metrics, backward, [all-reduce], clip+Adam — is captured into one
  HIP graph and replayed; validation/test steps are captured the same way.  The
  per-step host cost is one ``hipGraphLaunch``; nothing reads back to the host
  until the epoch ends.
"""
from __future__ import annotations

import os
import sys
import time
from pathlib import Path
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import torch

from ..metrics import Metric, sync_metrics
from ..ops.optim import FlatParameters, FusedAdam, set_producer_optimizer
from ..parallel import dist as pdist
from ..parallel.ddp import FlatDDP
from .callbacks import Callback, ModelCheckpoint, StepTimer
from ..utils.profiling import PhaseTimer, phase
from .checkpoint import (LIGHTNING_COMPAT_VERSION, atomic_save, capture_rng_states, load_checkpoint,
                         restore_rng_states)
from .schedulers import PlateauScheduler


def _batch_size(batch) -> int:
    return int(batch[0].shape[0]) if isinstance(batch, (list, tuple)) else int(batch.shape[0])


class _Graph:
    """A captured HIP graph; ``static_in`` is set when inputs are copied in (non-static loaders)."""

    def __init__(self, graph, out, static_in: Optional[Sequence[torch.Tensor]] = None):
        self.graph, self.out, self.static_in = graph, out, static_in

    def replay(self, batch=None):
        if self.static_in is not None and batch is not None:
            for s, b in zip(self.static_in, batch):
                if s.data_ptr() != b.data_ptr():
                    s.copy_(b, non_blocking=True)
        self.graph.replay()
        return self.out


def _group_sizes(events, skip_groups: int = 0):
    """(event pair, steps it covers) per step: a grouped graph's pair is repeated once per step it ran.  The first
    ``skip_groups`` launches (eager warm-up / capture groups) are dropped WHOLE, so a partially skipped group never
    divides its time by the wrong step count."""
    out = []
    for ev in events:
        if out and out[-1][0] is ev:
            out[-1][1] += 1
        else:
            out.append([ev, 1])
    if len(out) > skip_groups:
        out = out[skip_groups:]
    return [(ev, n) for ev, n in out for _ in range(n)]


class Trainer:
    def __init__(self, max_epochs: int = 1000, gradient_clip_val: Optional[float] = None,
                 precision: str = "32-true", enable_progress_bar: bool = True, enable_model_summary: bool = True,
                 logger=None, callbacks: Optional[List[Callback]] = None, check_val_every_n_epoch: int = 1,
                 num_sanity_val_steps: int = 2, accelerator: str = "auto", devices: Any = 1,
                 use_hip_graphs: bool = True, graph_warmup_steps: int = 2, matmul_precision: str = "high",
                 limit_train_batches: Optional[int] = None, limit_val_batches: Optional[int] = None,
                 limit_test_batches: Optional[int] = None, default_root_dir: str = ".",
                 max_steps: int = -1, fail_at_step: Optional[int] = None, deterministic: bool = False,
                 debug_serialize: bool = False,
                 log_every_n_steps: int = 50, steps_per_graph: int = 8, profiler: Optional[str] = None,
                 profile_steps: int = 20):
        self.max_epochs = int(max_epochs)
        self.max_steps = int(max_steps)
        self.gradient_clip_val = float(gradient_clip_val or 0.0)
        self.precision = str(precision)
        self.enable_progress_bar = enable_progress_bar
        self.enable_model_summary = enable_model_summary
        self.logger = logger
        self.callbacks: List[Callback] = list(callbacks or [])
        self.check_val_every_n_epoch = int(check_val_every_n_epoch or 1)
        self.num_sanity_val_steps = int(num_sanity_val_steps)
        self.accelerator = accelerator
        # ranks of this job (parallel/launch.py): "auto"/-1 = every visible GPU, an int = that many.  The configs'
        # trainer.devices is "auto" like Lightning's default; a programmatic Trainer defaults to 1 so that library
        # use (tests, notebooks) never re-runs its host script
        self.devices = devices
        self.use_hip_graphs = use_hip_graphs
        self.graph_warmup_steps = max(1, int(graph_warmup_steps))
        # consecutive training steps captured into ONE graph (device-resident loaders only): one graph launch per
        # S steps instead of per step — the ~19 us launch gap between back-to-back graph replays (r2 kernel
        # trace) is paid once per group.  Every step still runs in full (gather, fwd, decoder, bwd, optimizer).
        self.steps_per_graph = max(1, int(os.environ.get("MTA_STEPS_PER_GRAPH", steps_per_graph)))
        self.matmul_precision = matmul_precision
        self.limit_train_batches = limit_train_batches
        self.limit_val_batches = limit_val_batches
        self.limit_test_batches = limit_test_batches
        self.default_root_dir = default_root_dir
        env_fail = os.environ.get("MTA_FAIL_AT_STEP")
        self.fail_at_step = int(env_fail) if env_fail else fail_at_step
        # fault injection on the first MTA_FAIL_ATTEMPTS launcher attempts only (transient-failure tests)
        attempts = os.environ.get("MTA_FAIL_ATTEMPTS")
        if attempts is not None and int(os.environ.get("MTA_RETRY_ATTEMPT", "0")) >= int(attempts):
            self.fail_at_step = None
        self.heartbeat_file = os.environ.get("MTA_HEARTBEAT_FILE")
        # bit-reproducible runs: ordered weight-gradient reductions instead of f32 atomics (LSTM kernels), no
        # split-K atomics in the extras' GEMMs, block-ordered head-parameter partials (wide heads backward)
        self.deterministic = bool(deterministic) or os.environ.get("MTA_DETERMINISTIC", "0") == "1"
        # serialize / launch-blocking debug mode (utils/debug.py): synchronous launches, no captured graphs
        from ..utils.debug import apply_serialize_env, serialize_requested

        self.debug_serialize = serialize_requested(debug_serialize)
        if self.debug_serialize:
            apply_serialize_env()
            self.use_hip_graphs = False
            self.steps_per_graph = 1
        if self.deterministic:
            from ..ops import extras as _extras_op
            from ..ops import losses as _losses_op
            from ..ops import lstm as _lstm_op

            _lstm_op.set_deterministic(True)
            _losses_op.set_deterministic(True)
            if hasattr(_extras_op, "set_deterministic"):
                _extras_op.set_deterministic(True)
        # state
        self.current_epoch = 0
        self.global_step = 0
        self.callback_metrics: Dict[str, torch.Tensor] = {}
        self.logged_metrics: Dict[str, float] = {}
        self.sanity_checking = False
        self.should_stop = False
        self.num_val_batches = 0
        self.optimizer: Optional[FusedAdam] = None
        self.optimizer_name = "Adam"
        self.scheduler: Optional[PlateauScheduler] = None
        self.scheduler_cfg: Dict[str, Any] = {}
        self.flat: Optional[FlatParameters] = None
        self.ddp: Optional[FlatDDP] = None
        self.denv = pdist.get_env()
        self.device = torch.device("cpu")
        self.model = None
        self.datamodule = None
        self._graphs: Dict[Tuple, _Graph] = {}
        self._graph_loaders: Dict[int, Any] = {}  # keeps loaders alive while graphs key on id(loader)
        self._eager_counts: Dict[Tuple, int] = {}
        self._ones: Dict[Tuple, torch.Tensor] = {}
        # models exposing fused_training_step run it instead of training_step + backward (MTA_FUSED_STEP=0: off)
        self.fused_step = os.environ.get("MTA_FUSED_STEP", "1") != "0"
        self.step_timer = StepTimer()
        self.perf: Dict[str, float] = {}
        # tracing (utils/profiling.py): "phases" = eager steps with per-phase HIP-event timers (gather / fwd /
        # loss / bwd / allreduce / optim), "torch" = torch.profiler Chrome trace of the first profile_steps steps
        self.profiler = (os.environ.get("MTA_PROFILER") or profiler or None)
        if self.profiler not in (None, "phases", "torch"):
            raise ValueError(f"profiler must be None, 'phases' or 'torch', got {self.profiler!r}")
        self.profile_steps = int(profile_steps)
        self.phase_timer: Optional[PhaseTimer] = None
        self._torch_prof = None
        self._in_graph = False
        # keep the captured (un-instantiated) graphs for graph_census(): which node types each step graph holds
        self.keep_graphs = os.environ.get("MTA_KEEP_GRAPHS", "0") == "1"
        # MTA_DEBUG_FINITE=1: after every training step synchronise and name the first parameter whose local
        # (pre-sync) gradient or updated value is non-finite, with rank and step (localises a bad kernel / race)
        self.debug_finite = os.environ.get("MTA_DEBUG_FINITE", "0") == "1"
        self._dbg_step = 0
        self._dbg_reported = False

    # ------------------------------------------------------------------ properties
    @property
    def is_global_zero(self) -> bool:
        return self.denv.rank == 0

    @property
    def world_size(self) -> int:
        return self.denv.world_size

    @property
    def checkpoint_callback(self) -> Optional[ModelCheckpoint]:
        for c in self.callbacks:
            if isinstance(c, ModelCheckpoint):
                return c
        return None

    def _print(self, *a, **k) -> None:
        if self.is_global_zero:
            print(*a, **k, flush=True)

    # ------------------------------------------------------------------ setup
    def _launch_ranks(self) -> None:
        """Lightning's subprocess-script launch (`/root/reference/train.py:169-180` gets DDP from it implicitly):
        with ``devices`` > 1 and no rank environment yet, start ranks 1..N-1 re-running this script and become rank
        0 -- before anything touches the GPU (parallel/launch.py)."""
        from ..parallel import launch

        if launch.in_launched_job() or pdist._ENV is not None:
            return
        n = launch.resolve_devices(self.devices, self.accelerator)
        if n <= 1:
            return
        if os.environ.get("MTA_MULTIRUN_INPROC") == "1":
            if self.devices in ("auto", -1, "-1", None):
                return  # an in-process sequential sweep: one device per job (use hydra/launcher=gpu_pool for more)
            raise RuntimeError(f"trainer.devices={self.devices}: multi-process jobs cannot run inside an in-process "
                               "multirun; use hydra/launcher=gpu_pool (one GPU per trial) or a single run")
        launch.launch_script_ranks(n)

    def _setup_env(self) -> None:
        self._launch_ranks()
        want_cpu = self.accelerator == "cpu" or not torch.cuda.is_available()
        self.denv = pdist.init_distributed(device="cpu" if want_cpu else None)
        self.device = self.denv.device
        if self.logger is not None and hasattr(self.logger, "rank"):
            self.logger.rank = self.denv.rank
        for c in self.callbacks:
            if isinstance(c, ModelCheckpoint) and c.dirpath is None and self.logger is not None:
                c.dirpath = str(Path(self.logger.log_dir) / "checkpoints")

    def _setup_model(self, model) -> None:
        if self.model is not None and self.model is not model:
            # captured graphs hold the previous model's parameter / metric buffers: never replay them
            self._graphs.clear()
            self._eager_counts.clear()
            self._graph_loaders.clear()
        model.trainer = self
        model.to(self.device)
        model.matmul_precision = self._effective_matmul_precision()
        self.model = model

    def _effective_matmul_precision(self) -> str:
        if self.precision.startswith("bf16"):
            return "medium"
        return self.matmul_precision

    def _configure_optimizers(self, model) -> None:
        conf = model.configure_optimizers()
        opt, sched_cfg = conf, None
        if isinstance(conf, dict):
            opt, sched_cfg = conf["optimizer"], conf.get("lr_scheduler")
        elif isinstance(conf, (list, tuple)):
            opt = conf[0]
        self.flat = FlatParameters(model.parameters(), device=self.device)
        self.flat.names = [n for n, p in model.named_parameters() if p.requires_grad]
        g = opt.param_groups[0]
        adamw = isinstance(opt, torch.optim.AdamW)
        if not isinstance(opt, (torch.optim.Adam, torch.optim.AdamW)) or g.get("amsgrad"):
            raise NotImplementedError("the fused engine supports Adam / AdamW optimizers")
        self.optimizer = FusedAdam(self.flat, lr=g["lr"], betas=g["betas"], eps=g["eps"],
                                   weight_decay=g["weight_decay"], adamw=adamw)
        self.optimizer_name = "AdamW" if adamw else "Adam"
        self.scheduler_cfg = {}
        self.scheduler = None
        if sched_cfg is not None:
            sch = sched_cfg["scheduler"] if isinstance(sched_cfg, dict) else sched_cfg
            if isinstance(sch, torch.optim.lr_scheduler.ReduceLROnPlateau):
                self.scheduler = PlateauScheduler.from_torch(sch, self.optimizer)
            else:
                raise NotImplementedError("only ReduceLROnPlateau schedulers are supported")
            self.scheduler_cfg = {
                "monitor": sched_cfg.get("monitor", "loss/total/val") if isinstance(sched_cfg, dict) else None,
                "interval": sched_cfg.get("interval", "epoch") if isinstance(sched_cfg, dict) else "epoch",
                "frequency": int(sched_cfg.get("frequency", 1)) if isinstance(sched_cfg, dict) else 1,
            }
        self.ddp = FlatDDP(self.flat)
        self.ddp.broadcast_parameters()
        # gradient producers (weight-gradient GEMMs that overwrite their range and hand the clip norm its partials,
        # ops/optim.py): one process, or world > 1 with the xGMI all-reduce, whose kernel writes the clip norm's
        # partials of the REDUCED gradient (FlatDDP.norm_parts: the optimizer then reads no gradient for the norm).
        # The process group's all-reduce rewrites the buffer after the producers' partials: producers off there.
        self.grad_producers = self.ddp.world == 1 or self.ddp.norm_parts is not None
        set_producer_optimizer(self.optimizer if self.grad_producers else None)

    def _model_summary(self, model) -> None:
        if not (self.enable_model_summary and self.is_global_zero):
            return
        rows = []
        for name, mod in model.named_children():
            n = sum(p.numel() for p in mod.parameters())
            rows.append((name, type(mod).__name__, n))
        total = sum(p.numel() for p in model.parameters())
        train = sum(p.numel() for p in model.parameters() if p.requires_grad)
        print("  | Name" + " " * 12 + "| Type" + " " * 26 + "| Params")
        for i, (n, t, c) in enumerate(rows):
            print(f"{i} | {n:<16}| {t:<30}| {c:,}")
        print(f"{train:,} Trainable params\n{total - train:,} Non-trainable params\n{total:,} Total params")
        print(f"{total * 4 / 1e6:.3f} Total estimated model params size (MB)", flush=True)

    # ------------------------------------------------------------------ step machinery
    def _graphs_enabled(self) -> bool:
        return (self.use_hip_graphs and self.device.type == "cuda" and self.profiler != "phases"
                and getattr(self.model, "graph_capturable", True))

    def _allreduce_in_graph(self) -> bool:
        # the xGMI all-reduce (one- or two-shot) is a plain kernel: the whole step (sync + optimizer) is one graph.
        # RCCL stays outside unless MTA_GRAPH_ALLREDUCE=1 (graph capture of RCCL is not exercised here).
        return (self.ddp.world == 1 or getattr(self.ddp, "graph_safe", False)
                or os.environ.get("MTA_GRAPH_ALLREDUCE", "0") == "1")

    def _seed_grad(self, loss: torch.Tensor) -> torch.Tensor:
        # a persistent ones tensor: no fill node per step for autograd's implicit seed
        one = self._ones.get((loss.shape, loss.device, loss.dtype))
        if one is None:
            one = torch.ones_like(loss)
            self._ones[(loss.shape, loss.device, loss.dtype)] = one
        return one

    def _train_body(self, batch, batch_idx: int):
        """zero-grad, forward + fused loss, backward, [all-reduce], clip + Adam.

        The fused optimizer leaves the flat gradient zeroed, so a step that follows one needs no fill."""
        if not getattr(self.optimizer, "grads_zeroed", False):
            self.flat.grad.zero_()
        if self.ddp.world > 1 and (not self._in_graph or self._allreduce_in_graph()):
            self.ddp.begin_backward()  # arm the backward-overlapped gradient sync (parallel/overlap.py)
        fused = getattr(self.model, "fused_training_step", None)
        if fused is not None and self.fused_step and self.model.fused_step_supported(batch):
            loss = fused(batch, batch_idx)  # forward + decoder + backward without autograd
            if getattr(batch, "pending", False):
                raise RuntimeError("fused training step left a deferred batch gather unconsumed")
        else:
            if getattr(batch, "pending", False):
                batch.materialize()
            phase("fwd")
            loss = self.model.training_step(batch, batch_idx)
            phase("bwd")
            loss.backward(self._seed_grad(loss))
        if not self._in_graph or self._allreduce_in_graph():
            if self.ddp.world > 1:
                phase("allreduce")
            self._debug_check("local grad (eager)", self.flat.grad)
            self.ddp.allreduce_grads()
            self._debug_norm("summed grad", self.flat.grad)
            phase("optim")
            self.optimizer.step(self.gradient_clip_val, self.ddp.grad_scale, zero_grad=True,
                                ext_norm=self.ddp.norm_parts)
            self._debug_norm("optimizer", None)
        return loss

    def _after_graph(self) -> None:
        # world > 1: the RCCL all-reduce and the optimizer run outside the captured fwd/bwd graph
        if not self._allreduce_in_graph():
            self._debug_check("local grad (replayed graph)", self.flat.grad)
            self.ddp.allreduce_grads()
            self._debug_norm("summed grad", self.flat.grad)
            self.optimizer.step(self.gradient_clip_val, self.ddp.grad_scale, zero_grad=True,
                                ext_norm=self.ddp.norm_parts)
            self._debug_norm("optimizer", None)

    def _debug_norm(self, what: str, buf: Optional[torch.Tensor]) -> None:
        """MTA_DEBUG_FINITE: print the host fp64 norm of ``buf`` (or the optimizer's device norm) for early steps."""
        if not self.debug_finite or self._in_graph or self._dbg_step > 12:
            return
        if buf is None:
            torch.cuda.synchronize() if self.device.type == "cuda" else None
            v = float(self.optimizer.grad_norm.item())
        else:
            v = float(buf.detach().double().norm().item())
        print(f"[finite] rank {self.denv.rank} step {self._dbg_step}: {what} norm {v:.6g}", file=sys.stderr,
              flush=True)

    def _debug_check(self, what: str, buf: torch.Tensor) -> None:
        """MTA_DEBUG_FINITE: report (once) the first parameter range of ``buf`` holding a NaN/Inf."""
        if not self.debug_finite or self._dbg_reported or self._in_graph:
            return
        if what.startswith("local"):
            self._debug_norm(what, buf)
        torch.cuda.synchronize() if buf.is_cuda else None
        host = buf.detach().float().cpu()
        bad = ~torch.isfinite(host)
        if not bool(bad.any()):
            return
        names = getattr(self.flat, "names", None) or [f"param{i}" for i in range(len(self.flat.params))]
        for name, p, o in zip(names, self.flat.params, self.flat.offsets):
            n = int(bad[o:o + p.numel()].sum())
            if n:
                print(f"[finite] rank {self.denv.rank} step {self._dbg_step}: {what}: first non-finite range "
                      f"'{name}' ({n}/{p.numel()} elements)", file=sys.stderr, flush=True)
                break
        self._dbg_reported = True

    def _run(self, key: Tuple, provider: Callable[[], Sequence[torch.Tensor]], body: Callable, static: bool,
             warmup: int):
        """Run one step: eager for the first ``warmup`` calls of ``key``, then capture once and replay.

        ``provider`` returns the batch; when ``static`` it launches the in-graph gather into fixed
        buffers, otherwise it returns fresh tensors that are copied into the graph's inputs.
        """
        if not self._graphs_enabled():
            phase("gather")
            return body(provider())
        g = self._graphs.get(key)
        if g is None:
            n = self._eager_counts.get(key, 0)
            if n < warmup:
                self._eager_counts[key] = n + 1
                side = torch.cuda.Stream()
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    out = body(provider())
                torch.cuda.current_stream().wait_stream(side)
                return out
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph(keep_graph=self.keep_graphs) if self.keep_graphs else torch.cuda.CUDAGraph()
            if static:
                self._in_graph = True
                try:
                    with torch.cuda.graph(graph):
                        out = body(provider())
                finally:
                    self._in_graph = False
                g = _Graph(graph, out)
            else:
                batch = provider()
                static_in = [t.clone() for t in batch]
                self._in_graph = True
                try:
                    with torch.cuda.graph(graph):
                        out = body(static_in)
                finally:
                    self._in_graph = False
                g = _Graph(graph, out, static_in)
                self._graphs[key] = g
                out = g.replay(batch)
                return out
            self._graphs[key] = g
        if g.static_in is None:
            return g.replay()
        return g.replay(provider())

    def graph_census(self) -> Dict[Tuple, Dict[str, int]]:
        """Node types of every captured step graph (needs ``keep_graphs``): {graph key: {"kernel": n, "memset": n,
        "memcpy": n, "other": n}}.  The step graphs are meant to hold kernel nodes only (tests/test_gpu_graphs.py)."""
        from ..ops._lib import lib

        C = lib()
        names = {int(C.GRAPH_NODE_KERNEL): "kernel", int(C.GRAPH_NODE_MEMSET): "memset",
                 int(C.GRAPH_NODE_MEMCPY): "memcpy"}
        out = {}
        for key, g in self._graphs.items():
            counts = {"kernel": 0, "memset": 0, "memcpy": 0, "other": 0}
            for t in C.graph_node_types(int(g.graph.raw_cuda_graph())):
                counts[names.get(int(t), "other")] += 1
            out[key] = counts
        return out

    def _static_hooks(self, loader):
        """Streaming loaders stage batch ``s`` (H2D on their copy stream) before and fence after a step."""
        self._graph_loaders[id(loader)] = loader
        return getattr(loader, "before_static_step", None), getattr(loader, "after_static_step", None)

    def _train_step(self, loader, batch_idx: int, static: bool, batch=None):
        if static:
            B = loader.batch_size
            self.model._current_batch_size = B
            pre, post = self._static_hooks(loader)
            if pre is not None:
                pre()
            out = self._run(("train", B, True, id(loader)), lambda: self._gather_train(loader),
                            lambda b: self._train_body(b, batch_idx), True, self.graph_warmup_steps)
            if post is not None:
                post()
        else:
            B = _batch_size(batch)
            self.model._current_batch_size = B
            out = self._run(("train", B, False), lambda: batch, lambda b: self._train_body(b, batch_idx), False,
                            self.graph_warmup_steps)
        key = ("train", B, True, id(loader)) if static else ("train", B, False)
        if self._graphs_enabled() and key in self._graphs:
            self._after_graph()
        self._dbg_step += 1
        self._debug_check("parameters after the step", self.flat.data)
        return out

    def _can_group(self, loader) -> bool:
        """Whether training steps on ``loader`` may be captured S at a time: graphs on, an in-graph gather
        without per-step host hooks (device residency), the optimizer inside the graph."""
        if self.steps_per_graph <= 1 or not self._graphs_enabled() or not self._static_ok(loader):
            return False
        pre, post = self._static_hooks(loader)
        return pre is None and post is None and self._allreduce_in_graph()

    def _train_group(self, loader, batch_idx: int, S: int):
        """S consecutive training steps as one graph (see ``steps_per_graph``); each step gathers its own batch
        through the loader's device cursor."""
        B = loader.batch_size
        self.model._current_batch_size = B

        def body(first):
            out = self._train_body(first, batch_idx)
            for k in range(1, S):
                out = self._train_body(self._gather_train(loader), batch_idx + k)
            return out

        return self._run(("train", B, True, id(loader), S), lambda: self._gather_train(loader), body, True,
                         self.graph_warmup_steps)

    def _gather_train(self, loader):
        """Training batch from a static loader: the gather is deferred into the fused step's forward launch when
        the model folds it in (``accepts_deferred_gather``; one launch less per step), else the gather kernel."""
        defer = (self.fused_step and getattr(self.model, "accepts_deferred_gather", False)
                 and os.environ.get("MTA_DEFER_GATHER", "1") != "0")
        if defer:
            try:
                return loader.gather_static(defer=True)
            except TypeError:  # loaders without the deferred protocol (streaming ring)
                pass
        return loader.gather_static()

    def _eval_step(self, stage: str, loader, batch_idx: int, static: bool, batch=None):
        model = self.model
        fn = model.validation_step if stage == "val" else model.test_step
        if not getattr(model, "graph_capturable", True):
            # MIOpen's inference LSTM initialises hipBLASLt state on first use, which is illegal while a
            # stream is capturing: the reference-equivalent path evaluates eagerly
            if static:
                model._current_batch_size = loader.batch_size
                pre, post = self._static_hooks(loader)
                if pre is not None:
                    pre()
                out = fn(loader.gather_static(), batch_idx)
                if post is not None:
                    post()
                return out
            model._current_batch_size = _batch_size(batch)
            return fn(batch, batch_idx)
        if static:
            B = loader.batch_size
            model._current_batch_size = B
            pre, post = self._static_hooks(loader)
            if pre is not None:
                pre()
            out = self._run((stage, B, True, id(loader)), loader.gather_static, lambda b: fn(b, batch_idx), True, 1)
            if post is not None:
                post()
            return out
        B = _batch_size(batch)
        model._current_batch_size = B
        return self._run((stage, B, False), lambda: batch, lambda b: fn(b, batch_idx), False, 1)

    def _static_ok(self, loader) -> bool:
        return hasattr(loader, "supports_static") and loader.supports_static()

    def make_train_stepper(self, loader):
        """Callable running one training step per call on the loader's stream of batches (bench.py)."""
        static = self._static_ok(loader)
        state = {"epoch": -1, "left": 0, "i": 0, "it": None}

        group = self._can_group(loader)

        def step(n: int = 1):
            """Run ``n`` steps (n == steps_per_graph: one grouped graph when the epoch has room; else singly)."""
            out = None
            while n > 0:
                if state["left"] == 0:
                    state["epoch"] += 1
                    if static:
                        state["left"] = loader.begin_epoch(state["epoch"])
                    else:
                        loader.set_epoch(state["epoch"])
                        batches = [b for b in loader if _batch_size(b) == loader.batch_size]
                        state["it"] = iter(batches)
                        state["left"] = len(batches)
                S = self.steps_per_graph
                if group and n >= S and state["left"] >= S:
                    out = self._train_group(loader, state["i"] + 1, S)
                    state["left"] -= S
                    state["i"] += S
                    n -= S
                    continue
                state["left"] -= 1
                state["i"] += 1
                n -= 1
                if static:
                    out = self._train_step(loader, state["i"], True)
                else:
                    out = self._train_step(loader, state["i"], False, next(state["it"]))
            return out

        return step

    # ------------------------------------------------------------------ epoch helpers
    def _metrics_of(self, stage: str) -> Dict[str, Metric]:
        return self.model.logged_metrics(stage)

    def _compute_stage_metrics(self, stage: str) -> Dict[str, torch.Tensor]:
        ms = self._metrics_of(stage)
        sync_metrics(ms.values())
        out = {}
        for name, m in ms.items():
            out[name] = m.compute().detach().float().cpu()
        return out

    def _reset_stage_metrics(self, stage: str) -> None:
        for m in self._metrics_of(stage).values():
            m.reset()

    def log_metrics(self, metrics: Dict[str, float], step: int) -> None:
        vals = {k: float(v) for k, v in metrics.items()}
        self.logged_metrics.update(vals)
        if self.logger is not None and self.is_global_zero:
            self.logger.log_metrics(vals, step)

    def _limit(self, n: int, lim) -> int:
        if lim is None:
            return n
        if isinstance(lim, float) and lim <= 1.0:
            return max(1, int(n * lim))
        return min(n, int(lim))

    # ------------------------------------------------------------------ loops
    def _eval_loop(self, stage: str, loader, limit=None, epoch: int = 0) -> None:
        n_total = self._limit(len(loader), limit)
        if self._static_ok(loader):
            nfull = loader.begin_epoch(epoch)
            for i in range(min(nfull, n_total)):
                self._eval_step(stage, loader, i, True)
            if n_total > nfull:
                tail = loader.tail_batch()
                if tail is not None:
                    self._eval_step(stage, loader, nfull, False, tail)
            return
        for i, batch in enumerate(loader):
            if i >= n_total:
                break
            self._eval_step(stage, loader, i, False, batch)

    def heartbeat(self) -> None:
        """Touch the launcher's heartbeat file (hang detection of the gpu_pool / joblib child launchers)."""
        if self.heartbeat_file:
            try:
                with open(self.heartbeat_file, "w") as f:
                    f.write(f"{time.time()} {self.global_step}\n")
            except OSError:
                pass

    def _check_device_health(self) -> None:
        """Raise if a pipelined LSTM launch gave up on a hand-off, an xGMI all-reduce on a peer, or the single-launch
        clip+Adam on its grid-wide norm arrival (that step's update used a partial norm): their results were
        garbage."""
        if self.device.type == "cuda":
            from ..ops.lstm import check_pipeline_health
            from ..parallel.xgmi import check_all_health

            check_pipeline_health()
            check_all_health()
            st = getattr(self.optimizer, "sync_timeouts", None)
            if st is not None:
                n = int(st.item())
                if n:
                    st.zero_()
                    raise RuntimeError(f"fused clip+Adam: {n} grid-wide norm wait(s) gave up (those updates used a "
                                       "partial gradient norm)")

    def _run_eval(self, stage: str, loader, limit=None) -> Dict[str, torch.Tensor]:
        model = self.model
        model.eval()
        model._stage = "val" if stage == "sanity" else stage
        with torch.no_grad():
            self._eval_loop(model._stage, loader, limit)
        self._check_device_health()
        res = self._compute_stage_metrics(model._stage)
        self._reset_stage_metrics(model._stage)
        model.train()
        model._stage = "train"
        return res

    def _train_epoch(self, loader, epoch: int) -> Tuple[List[float], int]:
        """One epoch of training steps; returns per-step device times (ms) and samples per batch."""
        static = self._static_ok(loader)
        n_batches = self._limit(len(loader), self.limit_train_batches)
        cuda = self.device.type == "cuda"
        events: List[Tuple[Any, Any]] = []
        host_ms: List[float] = []
        B = loader.batch_size

        timer = self.phase_timer

        def timed(fn):
            if timer is not None:
                timer.begin_step()
                fn()
                timer.end_step()
                return
            if cuda:
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record()
                events.append((e0, e1))
            else:
                t0 = time.perf_counter()
                fn()
                host_ms.append((time.perf_counter() - t0) * 1e3)

        def pre_step(i):
            if self.profiler == "torch" and self.is_global_zero:
                self._torch_profile_tick()
            if self.fail_at_step is not None and self.global_step == self.fail_at_step:
                raise RuntimeError(f"fault injection: MTA_FAIL_AT_STEP={self.fail_at_step}")
            if self.heartbeat_file and i % 500 == 0:
                self.heartbeat()
            if self.enable_progress_bar and self.is_global_zero and (i % 500 == 0 or i == n_batches - 1):
                sys.stdout.write(f"\rEpoch {epoch}: {i + 1}/{n_batches}")
                sys.stdout.flush()

        if static:
            nfull = loader.begin_epoch(epoch)
            S = self.steps_per_graph if self._can_group(loader) else 1
            nrun = min(nfull, n_batches)
            i = 0
            while i < nrun:
                if 0 <= self.max_steps <= self.global_step:
                    break
                room = nrun - i
                if self.max_steps >= 0:
                    room = min(room, self.max_steps - self.global_step)
                fail_in = (self.fail_at_step is not None
                           and self.global_step <= self.fail_at_step < self.global_step + S)
                if S > 1 and room >= S and not fail_in:
                    for k in range(S):
                        pre_step(i + k)
                    first = i
                    n_ev = len(events)
                    timed(lambda: self._train_group(loader, first, S))
                    if cuda:  # one event pair per group: StepTimer gets S equal per-step shares
                        events.extend([events[n_ev]] * (S - 1))
                    i += S
                    self.global_step += S
                    continue
                pre_step(i)
                timed(lambda: self._train_step(loader, i, True))
                self.global_step += 1
                i += 1
            if n_batches > nfull and not (0 <= self.max_steps <= self.global_step):
                tail = loader.tail_batch()
                if tail is not None:
                    pre_step(nfull)
                    timed(lambda: self._train_step(loader, nfull, False, tail))
                    self.global_step += 1
        else:
            if hasattr(loader, "set_epoch"):
                loader.set_epoch(epoch)
            for i, batch in enumerate(loader):
                if i >= n_batches or (0 <= self.max_steps <= self.global_step):
                    break
                pre_step(i)
                B = _batch_size(batch)
                timed(lambda: self._train_step(loader, i, False, batch))
                self.global_step += 1
        if timer is not None:
            self.perf_phases = timer.summarize(skip=2)
            return [], B
        if cuda:
            torch.cuda.synchronize()
            host_ms = [a.elapsed_time(b) / n for (a, b), n in _group_sizes(events, self.graph_warmup_steps + 1)]
        if self.enable_progress_bar and self.is_global_zero:
            sys.stdout.write("\n")
        return host_ms, B

    def _print_devices(self) -> None:
        """Lightning's start-up device line (plus the GPU a pinned launcher trial was given)."""
        cuda = self.device.type == "cuda"
        extra = ""
        if cuda:
            extra = (f", device: {torch.cuda.get_device_name(self.device)}"
                     f" (HIP_VISIBLE_DEVICES={os.environ.get('HIP_VISIBLE_DEVICES', 'all')}, rank {self.denv.rank}"
                     f"/{self.denv.world_size})")
        self._print(f"GPU available: {torch.cuda.is_available()} (rocm), used: {cuda}{extra}")

    def fit(self, model, datamodule=None, ckpt_path: Optional[str] = None, train_dataloaders=None,
            val_dataloaders=None) -> None:
        try:
            self._fit(model, datamodule, ckpt_path, train_dataloaders, val_dataloaders)
        finally:
            # the gradient producers' overwrite semantics belong to this fit's optimizer only: a later manual
            # backward on the model (gradient checks, accumulation) must accumulate as usual
            set_producer_optimizer(None)

    def _fit(self, model, datamodule, ckpt_path, train_dataloaders, val_dataloaders) -> None:
        self._setup_env()
        self._print_devices()
        dm = datamodule
        self.datamodule = dm
        if dm is not None:
            dm.rank, dm.world_size, dm.device = self.denv.rank, self.denv.world_size, self.device
            if self.denv.local_rank == 0:
                dm.prepare_data()
            pdist.barrier()
            dm.setup("fit")
        self._setup_model(model)
        self._model_summary(model)
        self._configure_optimizers(model)
        start_epoch = 0
        if ckpt_path:
            start_epoch = self._restore(ckpt_path)
        for c in self.callbacks:
            c.on_fit_start(self, model)
        train_loader = train_dataloaders or dm.train_dataloader()
        val_loader = val_dataloaders or dm.val_dataloader()
        self.num_val_batches = self._limit(len(val_loader), self.limit_val_batches)

        if self.num_sanity_val_steps > 0 and start_epoch == 0:
            self.sanity_checking = True
            self._run_eval("sanity", val_loader, limit=self.num_sanity_val_steps)
            self.sanity_checking = False

        for epoch in range(start_epoch, self.max_epochs):
            self.current_epoch = epoch
            model._stage = "train"
            model.train()
            model.on_train_epoch_start()
            for c in self.callbacks:
                c.on_train_epoch_start(self, model)
            t_epoch = time.perf_counter()
            if self.profiler == "phases":
                self.phase_timer = PhaseTimer(self.device)
                with self.phase_timer:
                    step_ms, samples_per_batch = self._train_epoch(train_loader, epoch)
                self.phase_timer = None
            else:
                step_ms, samples_per_batch = self._train_epoch(train_loader, epoch)
            wall = time.perf_counter() - t_epoch
            perf = self.step_timer.summarize(step_ms, samples_per_batch, self.world_size)
            if self.profiler == "phases":
                perf.update(getattr(self, "perf_phases", {}))
                steps = sum(v for k, v in perf.items() if k.startswith("perf/phase/"))
                perf["perf/step_ms_p50"] = steps
                perf["perf/samples_per_s"] = samples_per_batch * self.world_size * 1000.0 / max(steps, 1e-9)
            perf["perf/epoch_wall_s"] = wall
            self.perf = perf
            nonfinite = float(self.optimizer.nonfinite.item())
            if nonfinite > 0:
                self._print(f"WARNING: {int(nonfinite)} step(s) with a non-finite gradient norm")
                self.optimizer.nonfinite.zero_()
            self._check_device_health()

            train_metrics = self._compute_stage_metrics("train")
            self._reset_stage_metrics("train")
            self.callback_metrics.update(train_metrics)
            log = {k: float(v) for k, v in train_metrics.items()}
            log["epoch"] = float(epoch)
            log.update(perf)
            self.log_metrics(log, step=max(self.global_step - 1, 0))

            if (epoch + 1) % self.check_val_every_n_epoch == 0 and self.num_val_batches > 0:
                val_metrics = self._run_eval("val", val_loader, limit=self.limit_val_batches)
                self.callback_metrics.update(val_metrics)
                vlog = {k: float(v) for k, v in val_metrics.items()}
                vlog["epoch"] = float(epoch)
                self.log_metrics(vlog, step=max(self.global_step - 1, 0))
                for c in self.callbacks:
                    c.on_validation_end(self, model)
            model.on_train_epoch_end()
            self.heartbeat()
            for c in self.callbacks:
                c.on_train_epoch_end(self, model)
            self._step_scheduler(epoch)
            summary = " ".join(f"{k}={float(v):.6g}" for k, v in self.callback_metrics.items())
            self._print(f"[epoch {epoch}] {summary} | step p50 {perf.get('perf/step_ms_p50', 0):.3f} ms, "
                        f"{perf.get('perf/samples_per_s', 0):.1f} samples/s")
            if self.should_stop or (0 <= self.max_steps <= self.global_step):
                break
        if self._torch_prof not in (None, False):  # fewer steps than profile_steps: export what was recorded
            self.global_step = max(self.global_step, self.graph_warmup_steps + 1 + self.profile_steps)
            self._torch_profile_tick()
        for c in self.callbacks:
            c.on_fit_end(self, model)
        if self.logger is not None:
            self.logger.finalize()

    def _torch_profile_tick(self) -> None:
        """profiler="torch": start at the first step after the graph warm-up, stop + export after
        ``profile_steps`` steps (Chrome trace in the logger's directory, else ``default_root_dir``)."""
        start = self.graph_warmup_steps + 1
        if self.global_step == start and self._torch_prof is None:
            acts = [torch.profiler.ProfilerActivity.CPU]
            if self.device.type == "cuda":
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self._torch_prof = torch.profiler.profile(activities=acts)
            self._torch_prof.start()
        elif self._torch_prof not in (None, False) and self.global_step >= start + self.profile_steps:
            if self.device.type == "cuda":
                torch.cuda.synchronize()
            self._torch_prof.stop()
            root = Path(self.logger.log_dir) if self.logger is not None else Path(self.default_root_dir)
            root.mkdir(parents=True, exist_ok=True)
            self.torch_trace_path = str(root / f"torch_trace_step{start}.json")
            self._torch_prof.export_chrome_trace(self.torch_trace_path)
            self._torch_prof = False  # done for this run

    def _step_scheduler(self, epoch: int) -> None:
        if self.scheduler is None:
            return
        freq = self.scheduler_cfg.get("frequency", 1)
        if (epoch + 1) % freq != 0:
            return
        mon = self.scheduler_cfg.get("monitor")
        if mon not in self.callback_metrics:
            raise KeyError(f"ReduceLROnPlateau conditioned on metric {mon} which is not available. "
                           f"Available metrics are: {sorted(self.callback_metrics)}")
        self.scheduler.step(float(self.callback_metrics[mon]))

    def validate(self, model, datamodule=None) -> Dict[str, float]:
        if self.model is None:
            self._setup_env()
            self._setup_model(model)
        dm = datamodule or self.datamodule
        if not dm.splits:
            dm.setup("fit")
        res = self._run_eval("val", dm.val_dataloader(), self.limit_val_batches)
        return {k: float(v) for k, v in res.items()}

    def test(self, model, datamodule=None) -> List[Dict[str, float]]:
        if self.model is None or self.model is not model:
            self._setup_env()
            self._setup_model(model)
        dm = datamodule or self.datamodule
        if dm is not None:
            dm.rank, dm.world_size, dm.device = self.denv.rank, self.denv.world_size, self.device
            if not dm.splits or dm.dataset is None:
                dm.setup("test")
        loader = dm.test_dataloader()
        model.eval()
        model._stage = "test"
        model.on_test_start()
        with torch.no_grad():
            self._eval_loop("test", loader, self.limit_test_batches)
        self._check_device_health()
        # sync every test-time Metric (logged or attribute) across ranks before on_test_end
        test_metrics = list(self._metrics_of("test").values())
        test_metrics += [m for name, m in model.named_children() if isinstance(m, Metric) and name.startswith("test")]
        sync_metrics(test_metrics)
        model.on_test_end()
        for c in self.callbacks:
            c.on_test_end(self, model)
        res = {k: float(v) for k, v in self._compute_stage_metrics("test").items()}
        self._reset_stage_metrics("test")
        model._stage = "train"
        if res:
            self.log_metrics(res, step=self.global_step)
        return [res]

    # ------------------------------------------------------------------ checkpointing
    def checkpoint_dict(self) -> Dict[str, Any]:
        model = self.model
        sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
        ck = {
            "epoch": self.current_epoch,
            "global_step": self.global_step,
            "pytorch-lightning_version": LIGHTNING_COMPAT_VERSION,
            "state_dict": sd,
            "loops": {"fit_loop": {"epoch_progress": {"current": {"completed": self.current_epoch + 1}},
                                   "epoch_loop.state_dict": {"_batches_that_stepped": self.global_step}}},
            "callbacks": {c.state_key: c.state_dict() for c in self.callbacks},
            "optimizer_states": [self.optimizer.state_dict()] if self.optimizer else [],
            "lr_schedulers": [self.scheduler.state_dict()] if self.scheduler else [],
            "hparams_name": "kwargs",
            "hyper_parameters": dict(model.hparams),
            "rng_states": capture_rng_states(),
            "mta": {"world_size": self.world_size, "precision": self.precision,
                    "matmul_precision": self._effective_matmul_precision(),
                    # non-persistent device RNG state (LSTM counter-hash dropout seeds): exact resume
                    "buffers": {k: v.detach().cpu().clone() for k, v in model.named_buffers()
                                if k.endswith("seeds")}},
        }
        model.on_save_checkpoint(ck)
        return ck

    def save_checkpoint(self, path) -> None:
        ck = self.checkpoint_dict() if self.is_global_zero else None
        if self.is_global_zero:
            atomic_save(ck, path)
        pdist.barrier()

    def _restore(self, path) -> int:
        ck = load_checkpoint(path, map_location="cpu")
        self.model.load_state_dict(ck["state_dict"])
        if ck.get("optimizer_states"):
            self.optimizer.load_state_dict(ck["optimizer_states"][0])
        if ck.get("lr_schedulers") and self.scheduler is not None:
            self.scheduler.load_state_dict(ck["lr_schedulers"][0])
        cbs = ck.get("callbacks", {})
        for c in self.callbacks:
            if c.state_key in cbs:
                c.load_state_dict(cbs[c.state_key])
        if "rng_states" in ck:
            restore_rng_states(ck["rng_states"])
        bufs = dict(self.model.named_buffers())
        for k, v in ck.get("mta", {}).get("buffers", {}).items():
            if k in bufs and bufs[k].shape == v.shape:
                bufs[k].copy_(v)
        self.global_step = int(ck.get("global_step", 0))
        self._print(f"Restored training state from {path} (epoch {ck['epoch']}, step {self.global_step})")
        return int(ck["epoch"]) + 1
