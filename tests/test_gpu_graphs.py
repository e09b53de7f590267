"""Audit of the captured training-step graphs: kernel nodes only.

The r3 multi-process NaN came from a captured ``hipMemsetAsync`` node that was not ordered against its neighbouring
kernel nodes when several processes shared the GPU (profiles/r4_nan_root_cause.txt).  Any memset or memcpy node in a
step graph is suspect for the same reason (a D2D copy node runs as the runtime's ``__amd_rocclr_copyBuffer`` blit
kernel), so every step graph the trainer captures -- LSTM (32-true), MLP and transformer (bf16-mixed), one step and
grouped steps per graph -- is walked node by node (``_C.graph_node_types``: hipGraphGetNodes / hipGraphNodeGetType,
child graphs recursively) and must hold kernel nodes only.  World 2 is covered in tests/test_gpu_dist_trainer.py.
"""
import os
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parents[1]


def _census(model: str, trainer: str, spg: int, loss: str = "mse", steps: int = 12):
    from masters_thesis_amd.config import compose
    from masters_thesis_amd.data import FinancialLstmDataModule
    from masters_thesis_amd.engine import Trainer
    from masters_thesis_amd.models import get_model_class, model_params_from_config

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cfg, _, _ = compose(REPO / "configs", "config", [f"model={model}", f"loss={loss}", f"trainer={trainer}",
                                                     "datamodule.n_samples=20000"])
    dm = FinancialLstmDataModule.from_config(cfg.datamodule, cache=False, device=dev)
    dm.setup("fit")
    net = get_model_class(cfg.loss.module_class, cfg.model.get("arch", "lstm"))(**model_params_from_config(cfg))
    tr = Trainer(max_epochs=1, gradient_clip_val=cfg.trainer.gradient_clip_val, precision=cfg.trainer.precision,
                 enable_progress_bar=False, enable_model_summary=False, logger=None, callbacks=[],
                 use_hip_graphs=True, steps_per_graph=spg)
    tr.keep_graphs = True
    tr._setup_env()
    tr._setup_model(net)
    tr._configure_optimizers(net)
    net.train()
    step = tr.make_train_stepper(dm.train_dataloader())
    done = 0
    while done < steps:
        n = spg if steps - done >= spg else 1
        step(n)
        done += n
    # a validation pass captures the eval-step graph too
    net.eval()
    net._stage = "val"
    with torch.no_grad():
        tr._eval_loop("val", dm.val_dataloader(), limit=4)
    torch.cuda.synchronize()
    assert tr.optimizer.nonfinite.item() == 0
    census = tr.graph_census()
    assert census, "no graph was captured"
    return census


@pytest.mark.parametrize("model,trainer,loss", [("small", "fast", "mse"), ("small", "fast", "combined"),
                                                ("mlp_small", "gpu_fast", "mse"),
                                                ("transformer_encoder", "gpu_fast", "combined")])
@pytest.mark.parametrize("spg", [1, 4])
def test_step_graphs_hold_kernel_nodes_only(model, trainer, loss, spg):
    census = _census(model, trainer, spg, loss)
    for key, c in census.items():
        print(f"[{model} spg={spg}] {key[:3]}: {c}")
    for key, c in census.items():
        assert c["kernel"] > 0, (key, c)
        assert c["memset"] == 0 and c["memcpy"] == 0 and c["other"] == 0, (key, c)
    if spg > 1:
        assert any(len(k) == 5 and k[-1] == spg for k in census), "no grouped graph was captured"


@pytest.mark.parametrize("model,trainer,limit", [("small", "fast", 4), ("transformer_encoder", "gpu_fast", 30)])
@pytest.mark.parametrize("spg", [1, 4])
def test_step_graph_launch_budget(model, trainer, limit, spg):
    """Kernel nodes per training step: the headline LSTM step is 4 launches (forward with the batch gather folded
    in, one-launch decoder, backward with the weight gradients, clip + Adam); the transformer_encoder step at most 30
    (fused attention / FFN halves, grouped weight gradients, embedding and operand casts folded in)."""
    census = _census(model, trainer, spg, "mse")
    per_step = max(c["kernel"] for c in census.values()) / spg
    assert per_step <= limit, (per_step, census)
