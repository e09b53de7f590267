"""Device-resident metrics (torchmetrics replacement).

Reference metrics: ``MeanSquaredError`` / ``MeanAbsoluteError`` (torchmetrics) and
the custom ``MultivariateGaussianNLLLoss`` with states ``loss_sum`` / ``total`` and
``dist_reduce_fx="sum"`` (`src/model.py:12-42`).

States are small device tensors updated in place (no host sync per step, so the
updates are captured inside the train-step HIP graph).  ``compute()`` reads them
once per epoch; ``sync()`` all-reduces every state of every metric in ONE fused
collective, instead of one all-gather per metric state.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional

import torch
from torch import Tensor


class Metric(torch.nn.Module):
    full_state_update = False
    is_differentiable = True
    higher_is_better = False

    def __init__(self):
        super().__init__()
        self._defaults: Dict[str, Tensor] = {}

    def add_state(self, name: str, default: Tensor, dist_reduce_fx: str = "sum") -> None:
        assert dist_reduce_fx == "sum", "only sum-reduced states are supported"
        self._defaults[name] = default.detach().clone()
        self.register_buffer(name, default.detach().clone(), persistent=False)

    def reset(self) -> None:
        for k in self._defaults:
            getattr(self, k).zero_()

    def state_tensors(self) -> List[Tensor]:
        return [getattr(self, k) for k in self._defaults]

    def update(self, *args) -> None:  # pragma: no cover - abstract
        raise NotImplementedError

    def compute(self) -> Tensor:  # pragma: no cover - abstract
        raise NotImplementedError


class MeanSquaredError(Metric):
    def __init__(self):
        super().__init__()
        self.add_state("sum_squared_error", torch.tensor(0.0, dtype=torch.float64))
        self.add_state("total", torch.tensor(0.0, dtype=torch.float64))

    @torch.no_grad()
    def update_from(self, sse: Tensor, count: int) -> None:
        self.sum_squared_error.add_(sse.detach().to(torch.float64))
        self.total.add_(count)

    @torch.no_grad()
    def update(self, preds: Tensor, target: Tensor) -> None:
        d = (preds - target).double()
        self.update_from((d * d).sum(), target.numel())

    def forward(self, preds: Tensor, target: Tensor) -> Tensor:
        d = preds - target
        val = (d * d).mean()
        self.update_from(val.detach() * target.numel(), target.numel())
        return val

    def compute(self) -> Tensor:
        return (self.sum_squared_error / self.total).float()


class MeanAbsoluteError(Metric):
    def __init__(self):
        super().__init__()
        self.add_state("sum_abs_error", torch.tensor(0.0, dtype=torch.float64))
        self.add_state("total", torch.tensor(0.0, dtype=torch.float64))

    @torch.no_grad()
    def update_from(self, sae: Tensor, count: int) -> None:
        self.sum_abs_error.add_(sae.detach().to(torch.float64))
        self.total.add_(count)

    @torch.no_grad()
    def update(self, preds: Tensor, target: Tensor) -> None:
        self.update_from((preds - target).abs().double().sum(), target.numel())

    def compute(self) -> Tensor:
        return (self.sum_abs_error / self.total).float()


class MultivariateGaussianNLLLoss(Metric):
    """Per-window NLL accumulator: ``loss_sum += nll, total += 1`` (`src/model.py:27-42`)."""

    def __init__(self):
        super().__init__()
        self.add_state("loss_sum", torch.tensor(0.0, dtype=torch.float64))
        self.add_state("total", torch.tensor(0.0, dtype=torch.float64))

    @torch.no_grad()
    def update_from(self, loss: Tensor, count: int = 1) -> None:
        self.loss_sum.add_(loss.detach().to(torch.float64))
        self.total.add_(count)

    @torch.no_grad()
    def update(self, mean: Tensor, inv_cov: Tensor, target: Tensor) -> None:
        from ..data.common import gaussian_nll_dense

        self.update_from(gaussian_nll_dense(mean, inv_cov, target))

    def compute(self) -> Tensor:
        return (self.loss_sum / self.total).float()

    @staticmethod
    def multivariate_gaussian_nll_loss(mean: Tensor, inv_cov: Tensor, target: Tensor) -> Tensor:
        from ..data.common import gaussian_nll_dense

        return gaussian_nll_dense(mean, inv_cov, target)


class MeanAccumulator(Metric):
    """Lightning's ``self.log(name, tensor, on_epoch=True)``: batch-size-weighted epoch mean."""

    def __init__(self):
        super().__init__()
        self.add_state("value_sum", torch.tensor(0.0, dtype=torch.float64))
        self.add_state("weight", torch.tensor(0.0, dtype=torch.float64))

    @torch.no_grad()
    def update(self, value: Tensor, weight: float = 1.0) -> None:
        self.value_sum.add_(value.detach().to(torch.float64) * weight)
        self.weight.add_(weight)

    def compute(self) -> Tensor:
        return (self.value_sum / self.weight).float()


class MetricAccumulator(Metric):
    """One float64[8] device buffer that the fused loss kernel adds into every step
    (``ops.losses.heads_losses(acc=...)``): [sse, count, nll_sum, nll_updates,
    total_sum, total_weight, sae, count].  The epoch metrics below are views of it, so
    the whole per-step metric bookkeeping costs zero extra kernels."""

    SSE, CNT, NLL, NLL_N, TOT, TOT_W, SAE, CNT2 = range(8)

    def __init__(self):
        super().__init__()
        self.add_state("acc", torch.zeros(8, dtype=torch.float64))


class _Linked(Metric):
    def __init__(self, source: MetricAccumulator, num: int, den: int):
        super().__init__()
        object.__setattr__(self, "_source", source)  # not a submodule: no duplicate state_dict/buffers
        self._num, self._den = num, den

    def state_tensors(self) -> List[Tensor]:
        return self._source.state_tensors()

    def reset(self) -> None:
        self._source.reset()

    def compute(self) -> Tensor:
        a = self._source.acc
        return (a[self._num] / a[self._den]).float()


class LinkedMSE(_Linked):
    def __init__(self, source: MetricAccumulator):
        super().__init__(source, MetricAccumulator.SSE, MetricAccumulator.CNT)


class LinkedNLL(_Linked):
    def __init__(self, source: MetricAccumulator):
        super().__init__(source, MetricAccumulator.NLL, MetricAccumulator.NLL_N)


class LinkedTotal(_Linked):
    def __init__(self, source: MetricAccumulator):
        super().__init__(source, MetricAccumulator.TOT, MetricAccumulator.TOT_W)


class LinkedMAE(_Linked):
    def __init__(self, source: MetricAccumulator):
        super().__init__(source, MetricAccumulator.SAE, MetricAccumulator.CNT2)


def sync_metrics(metrics: Iterable[Metric], group=None) -> None:
    """All-reduce (sum) every state of every metric in one flat collective."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    ms = list(metrics)
    seen = set()
    states = []
    for m in ms:
        for s in m.state_tensors():
            if s.data_ptr() not in seen:
                seen.add(s.data_ptr())
                states.append(s)
    if not states:
        return
    flat = torch.cat([s.reshape(-1).to(torch.float64) for s in states])
    if dist.get_backend(group) == "gloo" and flat.is_cuda:
        flat = flat.cpu()
    dist.all_reduce(flat, group=group)
    off = 0
    for s in states:
        n = s.numel()
        s.copy_(flat[off:off + n].reshape(s.shape).to(s.device, s.dtype))
        off += n


__all__ = ["Metric", "MeanSquaredError", "MeanAbsoluteError", "MultivariateGaussianNLLLoss", "MeanAccumulator",
           "MetricAccumulator", "LinkedMSE", "LinkedNLL", "LinkedTotal", "LinkedMAE", "sync_metrics"]
