"""Checkpoint evaluation + TensorBoard figures (reference `test.py:147-215`).

    python test.py checkpoint=logs/FinancialLstm/synthetic/<version>/checkpoints/last.ckpt [loss=... datamodule=...]

Runs the model and the OLS-on-lookback baseline (`test.py:41-72`) over the test
split and writes the scatter/histogram/estimation figures into the checkpoint's
TensorBoard run (`test.py:91-145`, tags in SURVEY.md A.3).  Evaluation runs on the
CPU like the reference unless ``+device=cuda`` is given.
"""
from __future__ import annotations

from pathlib import Path

import torch

from masters_thesis_amd.config import main as config_main, register_default_resolvers
from masters_thesis_amd.data import FinancialLstmDataModule
from masters_thesis_amd.data.common import ols
from masters_thesis_amd.models import get_model_class
from masters_thesis_amd.utils.logger import TensorBoardLogger
from masters_thesis_amd.utils.plots import estimation_plots, estimation_scatter, hist_plot, scatter_plot

register_default_resolvers()

_KINDS = ("recon_residuals", "alpha_residuals", "beta_residuals")


def init_test_results():
    res = {k: {"model": [], "ols": []} for k in _KINDS}
    res["alpha"] = {"model": [], "ols": [], "true": []}
    res["beta"] = {"model": [], "ols": [], "true": []}
    res["recon"] = {"model": [], "ols": [], "true": []}
    return res


def test_step(model, test_results, batch):
    context = batch[0].flatten(0, 1)
    target = batch[1].flatten(0, 1)
    r_target, r_market_target = target[:, :, 0], target[:, :, 1]
    alpha_target, beta_target = target[:, 0, 2], target[:, 0, 3]

    alpha_model, beta_model = model(context)
    alpha_ols, beta_ols = ols(context[0, :, 1], context[:, :, 0])  # OLS on the LOOKBACK window

    r_pred_model = alpha_model + beta_model * r_market_target
    r_pred_ols = alpha_ols.unsqueeze(-1) + beta_ols.unsqueeze(-1) * r_market_target
    alpha_model, beta_model = alpha_model.squeeze(-1), beta_model.squeeze(-1)

    tr = test_results
    tr["recon_residuals"]["model"].append((r_target - r_pred_model).detach())
    tr["alpha_residuals"]["model"].append((alpha_target - alpha_model).detach())
    tr["beta_residuals"]["model"].append((beta_target - beta_model).detach())
    tr["recon_residuals"]["ols"].append((r_target - r_pred_ols).detach())
    tr["alpha_residuals"]["ols"].append((alpha_target - alpha_ols).detach())
    tr["beta_residuals"]["ols"].append((beta_target - beta_ols).detach())
    tr["recon"]["model"].append(r_pred_model.detach().flatten())
    tr["recon"]["ols"].append(r_pred_ols.detach().flatten())
    tr["recon"]["true"].append(r_target.detach().flatten())
    for k, m, o, t in (("alpha", alpha_model, alpha_ols, alpha_target), ("beta", beta_model, beta_ols, beta_target)):
        tr[k]["model"].append(m.detach())
        tr[k]["ols"].append(o.detach())
        tr[k]["true"].append(t.detach())


def transform_test_results(tr):
    for src in ("model", "ols"):
        tr["recon_residuals"][src] = torch.stack(tr["recon_residuals"][src]).mean(dim=-1).cpu()
        tr["alpha_residuals"][src] = torch.stack(tr["alpha_residuals"][src]).cpu()
        tr["beta_residuals"][src] = torch.stack(tr["beta_residuals"][src]).cpu()
    for k in ("alpha", "beta", "recon"):
        for src in ("model", "ols", "true"):
            tr[k][src] = torch.stack(tr[k][src]).cpu()


def _corr(a, b) -> float:
    return float(torch.corrcoef(torch.stack([a.flatten().double(), b.flatten().double()]))[0, 1])


def summary(tr) -> dict:
    """The thesis' estimation correlations (`tex/diplomski_rad.tex:1193-1212`): alpha / beta estimates and the
    return reconstruction of the model and of OLS-on-lookback against the truth, and model vs OLS."""
    out = {}
    for k in ("alpha", "beta", "recon"):
        m, o, t = tr[k]["model"], tr[k]["ols"], tr[k]["true"]
        out[f"{k}_corr_model"] = _corr(m, t)
        out[f"{k}_corr_ols"] = _corr(o, t)
        out[f"{k}_corr_model_vs_ols"] = _corr(m, o)
    out["n_test_windows"] = int(tr["alpha"]["model"].shape[0])
    return out


def plot(tb_logger, tr):
    tr = {k: v for k, v in tr.items() if k != "recon"}
    tb = tb_logger.experiment
    tb.add_figure("scatter/recon_residuals", scatter_plot(tr["recon_residuals"]["model"], tr["recon_residuals"]["ols"],
                                                          title="Model vs OLS Reconstruction Residuals"))
    tb.add_figure("scatter/alphas", scatter_plot(tr["alpha"]["model"], tr["alpha"]["ols"], title="Model vs OLS Alphas"))
    tb.add_figure("scatter/betas", scatter_plot(tr["beta"]["model"], tr["beta"]["ols"], title="Model vs OLS Betas"))
    tb.add_figure("hist/recon_residuals", hist_plot(tr["recon_residuals"]["model"], tr["recon_residuals"]["ols"],
                                                    title="Model vs OLS Reconstruction Residuals"))
    tb.add_figure("hist/alphas", hist_plot(tr["alpha_residuals"]["model"], tr["alpha_residuals"]["ols"],
                                           title="Model vs OLS Alpha Residuals"))
    tb.add_figure("hist/betas", hist_plot(tr["beta_residuals"]["model"], tr["beta_residuals"]["ols"],
                                          title="Model vs OLS Beta Residuals"))
    estimation_plots(tb, tr["alpha"]["model"], tr["alpha"]["ols"], tr["alpha"]["true"], est_kind="alpha")
    estimation_plots(tb, tr["beta"]["model"], tr["beta"]["ols"], tr["beta"]["true"], est_kind="beta")
    tb.add_figure("estimation/alpha", estimation_scatter(tr["alpha"]["model"], tr["alpha"]["ols"],
                                                         tr["alpha"]["true"], est_kind="alpha"))
    tb.add_figure("estimation/beta", estimation_scatter(tr["beta"]["model"], tr["beta"]["ols"], tr["beta"]["true"],
                                                        est_kind="beta"))


def tb_location(checkpoint: Path):
    """save_dir / name / version from the checkpoint path (`test.py:182-192`, absolute paths handled: Q19)."""
    parts = checkpoint.parts
    if "checkpoints" in parts:
        i = len(parts) - 1 - parts[::-1].index("checkpoints")
        version = parts[i - 1]
        name = "/".join(parts[i - 3:i - 1])
        save_dir = str(Path(*parts[:i - 3])) if i - 3 > 0 else "."
        return save_dir, name, version
    return parts[0], "/".join(parts[1:3]), parts[3]


@config_main(version_base=None, config_path="configs", config_name="config")
def main(cfg):
    if not cfg.checkpoint:
        print("No checkpoint provided")
        return

    print("\n" + "=" * 70)
    print("EXPERIMENT CONFIGURATION")
    print("=" * 70)
    print(f"Datamodule: {cfg.datamodule.name}")
    print(f"Model: {cfg.model.name}")
    print(f"Checkpoint: {cfg.checkpoint}")
    print("=" * 70 + "\n")

    device = torch.device(cfg.get("device", "cpu"))
    dm = FinancialLstmDataModule.from_config(cfg.datamodule, device=device)
    ModelClass = get_model_class(cfg.loss.module_class, cfg.model.get("arch", "lstm"))
    model = ModelClass.load_from_checkpoint(cfg.checkpoint, map_location="cpu").to(device)
    print(model)

    save_dir, name, version = tb_location(Path(cfg.checkpoint))
    tb_logger = TensorBoardLogger(save_dir=save_dir, name=name, version=version, default_hp_metric=False)

    print("\n" + "=" * 50)
    print("Starting Testing...")
    print("=" * 50 + "\n")
    dm.prepare_data()
    dm.setup("test")
    test_loader = dm.test_dataloader()
    results = init_test_results()
    model.eval()
    with torch.no_grad():
        for batch in test_loader:
            test_step(model, results, batch)
    transform_test_results(results)
    plot(tb_logger, results)
    tb_logger.close()
    import json

    print("[test-summary] " + json.dumps(summary(results)), flush=True)

    print("\n" + "=" * 50)
    print("Testing and plotting Complete!")
    print("=" * 50)
    return results


if __name__ == "__main__":
    main()
