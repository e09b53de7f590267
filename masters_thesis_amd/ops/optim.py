"""Flat-buffer parameters and the fused clip + Adam/AdamW optimizer.

Reference: ``torch.optim.Adam(params, lr, weight_decay)`` (coupled L2,
`src/model.py:150-154`) preceded by Lightning's ``gradient_clip_val`` norm clipping
(`train.py:171`, `configs/trainer/*.yaml:2`).

MI355X design:

* ``FlatParameters`` moves every parameter (and its gradient) into ONE contiguous
  fp32 buffer, padded to a multiple of 1024 floats.  Each ``param.data`` /
  ``param.grad`` becomes a view, so autograd accumulates straight into the flat
  gradient buffer — which is then the single DDP all-reduce bucket (one RCCL call
  per step for the <= 1 MB gradients of this workload) and the single input of
  the fused optimizer.
* ``FusedAdam.step`` is ONE HIP launch (``csrc/optim.hip:adam_fused_kernel``): per-workgroup
  partial grad norms, an in-launch arrival ticket (write-through partials, no fences), then
  clip + Adam with ``lr`` and the step counter in device memory, i.e. it can be captured once
  in a HIP graph and replayed forever; the plateau scheduler only writes the lr scalar.  With
  ``zero_grad=True`` the kernel leaves the gradient zeroed, which replaces the per-step fill
  (``grads_zeroed`` tells the trainer).  ``single_launch=False`` selects the older
  norm + update pair (slower: profiles/r5_adam_two_launch_ab.jsonl; kept as the test oracle).
"""
from __future__ import annotations

import math
import os
from typing import Dict, Iterable, List, Optional

import torch
from torch import Tensor

from ._lib import lib, use_hip

_ALIGN = 1024

# The optimizer whose flat gradient the ops may produce into by OVERWRITING (see FusedAdam.register_producer), or None.
_PRODUCER_OPT: List[Optional["FusedAdam"]] = [None]


def set_producer_optimizer(opt: Optional["FusedAdam"]) -> None:
    """Enable (single-process training) or disable gradient producers for ``opt`` (the trainer calls this)."""
    _PRODUCER_OPT[0] = opt


def register_grad_producer(grad: Tensor) -> Optional[Tensor]:
    """For a weight-gradient op about to write ``grad`` (a view into the active optimizer's flat gradient): the norm
    partials buffer it must fill, with overwrite semantics (``lib().gemm_grad_producer(parts, True)``), or None
    (accumulate as usual)."""
    opt = _PRODUCER_OPT[0]
    return None if opt is None else opt.register_producer(grad)


class FlatParameters:
    def __init__(self, params: Iterable[torch.nn.Parameter], device: Optional[torch.device] = None):
        self.params: List[torch.nn.Parameter] = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("no trainable parameters")
        dev = device or self.params[0].device
        self.offsets: List[int] = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            # every parameter starts on a 16-byte boundary: its range is whole float4s (the vectorised kernels and
            # the gradient producers' covered ranges); the gaps stay zero in every buffer
            off += -(-p.numel() // 4) * 4
        self.numel = off
        self.padded = -(-off // _ALIGN) * _ALIGN
        self.data = torch.zeros(self.padded, device=dev, dtype=torch.float32)
        self.grad = torch.zeros(self.padded, device=dev, dtype=torch.float32)
        for p, o in zip(self.params, self.offsets):
            n = p.numel()
            self.data[o:o + n].copy_(p.detach().reshape(-1).to(dev, torch.float32))
            p.data = self.data[o:o + n].view_as(p)
            p.grad = self.grad[o:o + n].view_as(p)

    def zero_grad(self) -> None:
        self.grad.zero_()

    def ensure_grad_views(self) -> None:
        """Re-attach grad views if something replaced ``p.grad`` (e.g. set_to_none)."""
        for p, o in zip(self.params, self.offsets):
            n = p.numel()
            if p.grad is None or p.grad.data_ptr() != self.grad[o:o + n].data_ptr():
                if p.grad is not None:
                    self.grad[o:o + n].copy_(p.grad.reshape(-1))
                p.grad = self.grad[o:o + n].view_as(p)

    def views(self, buf: Tensor) -> List[Tensor]:
        return [buf[o:o + p.numel()].view_as(p) for p, o in zip(self.params, self.offsets)]


class FusedAdam:
    """Adam (coupled L2, torch.optim.Adam semantics) or AdamW over a FlatParameters buffer."""

    def __init__(self, flat: FlatParameters, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, adamw: bool = False, single_launch: bool = True):
        self.flat = flat
        dev = flat.data.device
        self.exp_avg = torch.zeros_like(flat.data)
        self.exp_avg_sq = torch.zeros_like(flat.data)
        self.lr_t = torch.tensor([lr], device=dev, dtype=torch.float32)
        self.step_t = torch.zeros(1, device=dev, dtype=torch.float32)
        self.grad_norm = torch.zeros(1, device=dev, dtype=torch.float32)
        # [0] steps with a NaN/Inf grad norm, [1] in-launch arrival waits that gave up (fused kernel)
        self._health = torch.zeros(2, device=dev, dtype=torch.float32)
        self.nonfinite = self._health[0:1]
        self.sync_timeouts = self._health[1:2]
        self.grads_zeroed = False  # True after a step that left the flat gradient zeroed
        self.betas = tuple(float(b) for b in betas)
        self.eps = float(eps)
        self.weight_decay = float(weight_decay)
        self.adamw = bool(adamw)
        self._lr = float(lr)
        self.hip = use_hip(flat.data)
        # gradient producers (register_producer): float4 ranges of the flat gradient a weight-gradient GEMM overwrote
        # this step, and their clip-norm partials; consumed by the next step()
        self._plan: Dict[tuple, tuple] = {}
        self._dropped: set = set()  # ranges produced twice this step: accumulated, not covered
        if self.hip:
            C = lib()
            self.single_launch = bool(single_launch)
            n = C.adam_fused_partials() if self.single_launch else C.optim_num_partials(flat.padded)
            self.partials = torch.zeros(n, device=dev, dtype=torch.float32)
            self.ticket = torch.zeros(1, device=dev, dtype=torch.int64)
            self._nparts = int(C.gemm_norm_parts())
            self.ext_parts = torch.zeros(self.MAX_PRODUCERS * self._nparts, device=dev, dtype=torch.float32)
        # torch.optim-like surface for schedulers / LR monitors / checkpoints
        self.param_groups = [{
            "lr": lr, "betas": self.betas, "eps": self.eps, "weight_decay": self.weight_decay, "amsgrad": False,
            "maximize": False, "foreach": None, "capturable": True, "differentiable": False, "fused": True,
            "decoupled_weight_decay": self.adamw, "params": list(range(len(flat.params))),
        }]

    MAX_PRODUCERS = 8  # csrc/optim.hip MAX_COVERED

    def register_producer(self, grad: Tensor) -> Optional[Tensor]:
        """A producer that overwrites ``grad`` (contiguous view into the flat gradient, float4-aligned) and writes the
        clip-norm partials of it into the returned buffer; this step's fused update then neither re-reads it for the
        norm nor zeroes it.  None when not applicable (accumulate as usual).  Decided from static properties only
        (alignment, slots), so a producer makes the same choice every step: a range the update left unzeroed is
        always overwritten by the next backward."""
        if not (self.hip and self.single_launch) or os.environ.get("MTA_OPTIM_PRODUCERS", "1") == "0":
            return None
        f = self.flat
        if not grad.is_contiguous() or grad.dtype != torch.float32:
            return None
        off = (grad.data_ptr() - f.grad.data_ptr()) // 4
        n = grad.numel()
        if off < 0 or off + n > f.padded or off % 4 or n % 4:
            return None
        key = (off // 4, (off + n) // 4)
        clash = [k for k in self._plan if k[0] < key[1] and key[0] < k[1]]
        if clash:
            # a second producer of the same range before step() (a weight used twice, two backward calls): the
            # first one overwrote the range, this one must ADD to it, and the range's norm partials would be stale
            # -- drop the range from this step's covered plan (the update re-reads it for the norm and zeroes it)
            # and let this GEMM accumulate
            for k in clash:
                del self._plan[k]
                self._dropped.add(k)
            self._dropped.add(key)
            return None
        if any(k[0] < key[1] and key[0] < k[1] for k in self._dropped):
            return None
        used = {s for _, _, s in self._plan.values()}
        free = [s for s in range(self.MAX_PRODUCERS) if s not in used]
        if not free:
            return None
        self._plan[key] = (key[0], key[1], free[0])
        slot = free[0]
        return self.ext_parts[slot * self._nparts:(slot + 1) * self._nparts]

    # ---- lr (device-resident) --------------------------------------------------
    @property
    def lr(self) -> float:
        return self._lr

    def set_lr(self, lr: float) -> None:
        self._lr = float(lr)
        self.param_groups[0]["lr"] = float(lr)
        self.lr_t.fill_(float(lr))

    def sync_lr_from_groups(self) -> None:
        if self.param_groups[0]["lr"] != self._lr:
            self.set_lr(self.param_groups[0]["lr"])

    # ---- step -------------------------------------------------------------------
    def step(self, max_norm: float = 0.0, grad_scale: float = 1.0, zero_grad: bool = False,
             ext_norm: Optional[Tensor] = None) -> None:
        """Clip (if max_norm > 0) the flat gradient scaled by ``grad_scale`` and apply one Adam step.

        ``zero_grad``: leave the flat gradient zeroed (the fused kernel writes 0 instead of the clipped
        gradient; ``grads_zeroed`` reports whether that happened).  ``ext_norm``: partial sums of squares of the
        WHOLE gradient written by its producer (world > 1: the xGMI all-reduce kernel, ``FlatDDP.norm_parts``): the
        fused kernel takes the clip norm from them instead of re-reading the gradient, and the producers' ranges only
        stay unzeroed."""
        self.sync_lr_from_groups()
        f = self.flat
        b1, b2 = self.betas
        self.grads_zeroed = False
        if self.hip and self.single_launch:
            plan = sorted(self._plan.values(), key=lambda r: r[2])
            self._plan = {}
            self._dropped = set()
            ext = None
            if ext_norm is not None:
                # the producers' own partials are of the local gradient (the all-reduce rewrote their ranges): unused
                lib().adam_fused(f.data, f.grad, self.exp_avg, self.exp_avg_sq, self.partials, self.ticket, self.lr_t,
                                 self.step_t, b1, b2, self.eps, self.weight_decay, float(max_norm or 0.0),
                                 float(grad_scale), self.adamw, bool(zero_grad), self.grad_norm, self._health,
                                 [r[0] for r in plan], [r[1] for r in plan], ext_norm, True)
                self.grads_zeroed = bool(zero_grad)
                return
            if plan:
                # the kernel sums every partial of ext: hand it slots [0, last used] and zero the slots in between
                # that no covered range owns (a range dropped by a double registration left its stale partials there)
                top = plan[-1][2] + 1
                used = {r[2] for r in plan}
                for s in range(top):
                    if s not in used:
                        self.ext_parts[s * self._nparts:(s + 1) * self._nparts].zero_()
                ext = self.ext_parts[:top * self._nparts]
            lib().adam_fused(f.data, f.grad, self.exp_avg, self.exp_avg_sq, self.partials, self.ticket, self.lr_t,
                             self.step_t, b1, b2, self.eps, self.weight_decay, float(max_norm or 0.0),
                             float(grad_scale), self.adamw, bool(zero_grad), self.grad_norm, self._health,
                             [r[0] for r in plan], [r[1] for r in plan], ext, False)
            # covered ranges keep this step's gradient (their producers overwrite them next step)
            self.grads_zeroed = bool(zero_grad)
            return
        if self.hip:
            C = lib()
            C.grad_sqnorm(f.grad, float(grad_scale), self.partials, self.step_t)
            C.adam(f.data, f.grad, self.exp_avg, self.exp_avg_sq, self.partials, self.lr_t, self.step_t, b1, b2,
                   self.eps, self.weight_decay, float(max_norm or 0.0), float(grad_scale), self.adamw,
                   self.grad_norm, self.nonfinite)
            return
        self._step_torch(max_norm, grad_scale)

    @torch.no_grad()
    def _step_torch(self, max_norm: float, grad_scale: float) -> None:
        f = self.flat
        b1, b2 = self.betas
        g = f.grad
        if grad_scale != 1.0:
            g.mul_(grad_scale)
        # clip_grad_norm_ semantics: norm over all grads, coef = max_norm / (norm + 1e-6), clamp 1
        norms = torch.stack([v.norm() for v in f.views(g)])
        total = norms.norm()
        self.grad_norm.copy_(total.reshape(1))
        if not torch.isfinite(total):
            self.nonfinite += 1
        if max_norm and max_norm > 0:
            coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
            g.mul_(coef)
        self.step_t += 1
        t = float(self.step_t.item())
        lr = self._lr
        p, m, v = f.data, self.exp_avg, self.exp_avg_sq
        if self.adamw:
            p.mul_(1 - lr * self.weight_decay)
            gg = g
        else:
            gg = g.add(p, alpha=self.weight_decay) if self.weight_decay else g
        m.lerp_(gg, 1 - b1)
        v.mul_(b2).addcmul_(gg, gg, value=1 - b2)
        bc1 = 1 - b1 ** t
        bc2 = 1 - b2 ** t
        denom = (v.sqrt() / math.sqrt(bc2)).add_(self.eps)
        p.addcdiv_(m, denom, value=-lr / bc1)

    def zero_grad(self, set_to_none: bool = False) -> None:
        self.flat.zero_grad()

    # ---- torch.optim.Adam-compatible state dict (Lightning 'optimizer_states') -----
    def state_dict(self) -> Dict:
        step = self.step_t.detach().cpu().reshape(())
        state = {}
        for i, (mv, vv) in enumerate(zip(self.flat.views(self.exp_avg), self.flat.views(self.exp_avg_sq))):
            state[i] = {"step": step.clone(), "exp_avg": mv.detach().cpu().clone(),
                        "exp_avg_sq": vv.detach().cpu().clone()}
        groups = [dict(self.param_groups[0])]
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, sd: Dict) -> None:
        g = sd["param_groups"][0]
        self.betas = tuple(g.get("betas", self.betas))
        self.eps = g.get("eps", self.eps)
        self.weight_decay = g.get("weight_decay", self.weight_decay)
        self.set_lr(g["lr"])
        mvs = self.flat.views(self.exp_avg)
        vvs = self.flat.views(self.exp_avg_sq)
        step = 0.0
        for i, st in sd["state"].items():
            i = int(i)
            mvs[i].copy_(st["exp_avg"].to(mvs[i].device))
            vvs[i].copy_(st["exp_avg_sq"].to(vvs[i].device))
            step = float(st["step"])
        self.step_t.fill_(step)
