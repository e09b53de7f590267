"""Trace the optimizer gradient-producer bookkeeping through a Trainer step (eager, then captured), on the GPU:
which weight gradients registered as producers, the plan each step consumed and what ext_parts holds afterwards."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
os.environ["MTA_OPTIM_PRODUCERS"] = "1"

from masters_thesis_amd.data.datamodule import TensorBatchLoader  # noqa: E402
from masters_thesis_amd.engine import Trainer  # noqa: E402
from masters_thesis_amd.models import get_model_class  # noqa: E402
from masters_thesis_amd.ops import optim as O  # noqa: E402

DEV = torch.device("cuda:0")
calls = []
orig_reg = O.FusedAdam.register_producer


def reg(self, grad):
    r = orig_reg(self, grad)
    calls.append((tuple(grad.shape), r is not None))
    return r


O.FusedAdam.register_producer = reg
orig_step = O.FusedAdam.step


def step(self, *a, **k):
    print(f"  step: plan={sorted(self._plan.values(), key=lambda r: r[2])} calls={calls}", flush=True)
    calls.clear()
    return orig_step(self, *a, **k)


O.FusedAdam.step = step

for graphs in (False, True):
    g = torch.Generator().manual_seed(0)
    W = 64
    data = [torch.randn(W, 100, 60, 3, generator=g), torch.randn(W, 100, 30, 4, generator=g) * 0.01,
            torch.stack([torch.randn(W, generator=g) * 0.01, torch.rand(W, generator=g) * 1e-3 + 1e-4], -1),
            torch.rand(W, 100, generator=g) * 3 + 1]
    torch.manual_seed(1)
    model = get_model_class("FinancialLstmMse", "mlp")(input_size=3, hidden_size=1024, num_layers=3, dropout=0.0,
                                                         learning_rate=1e-3)
    tr = Trainer(gradient_clip_val=0.05, enable_progress_bar=False, enable_model_summary=False,
                 use_hip_graphs=graphs, precision="bf16-mixed")
    tr._setup_env()
    tr._setup_model(model)
    tr._configure_optimizers(model)
    print(f"graphs={graphs} producer opt set: {O._PRODUCER_OPT[0] is tr.optimizer} hip={tr.optimizer.hip} "
          f"single={getattr(tr.optimizer, 'single_launch', None)}", flush=True)
    model.train()
    stepper = tr.make_train_stepper(TensorBatchLoader([t.to(DEV) for t in data], 1, shuffle=True, seed=0))
    for i in range(4):
        stepper()
        torch.cuda.synchronize()
        print(f"  after step {i}: ext_parts sum {tr.optimizer.ext_parts.abs().sum().item():.4g} "
              f"grad norm {tr.optimizer.grad_norm.item():.4g}", flush=True)
