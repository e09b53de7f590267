"""Evaluation figures written to TensorBoard by ``test.py`` (reference `src/plots.py:1-111`).

* ``scatter_plot``      model vs OLS values with identity line and Pearson correlation;
* ``hist_plot``         overlaid density histograms with mean / std markers;
* ``estimation_plots``  up to 9 per-stock time series, one figure per stock as steps of
  the ``estimation/examples_<kind>`` tag;
* ``estimation_scatter`` two panels: ground truth vs model and vs OLS.
All figures are 16 x 9 inches like the reference.
"""
from __future__ import annotations

import matplotlib

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402
from torch import Tensor  # noqa: E402

FIGSIZE = (16, 9)


def _corr(a: Tensor, b: Tensor) -> float:
    return float(torch.corrcoef(torch.stack([a.flatten().double(), b.flatten().double()]))[0, 1])


def scatter_plot(model: Tensor, ols: Tensor, title: str):
    fig = plt.figure(figsize=FIGSIZE)
    m, o = model.flatten(), ols.flatten()
    plt.scatter(m.numpy(), o.numpy(), marker=".")
    plt.xlabel("Model")
    plt.ylabel("OLS")
    lims = (float(m.min()), float(m.max()))
    plt.plot(lims, lims, "r--")
    plt.title(f"{title}, corr={_corr(m, o):.4f}")
    plt.grid(alpha=0.5)
    return fig


def hist_plot(model: Tensor, ols: Tensor, title: str):
    fig = plt.figure(figsize=FIGSIZE)
    m, o = model.flatten(), ols.flatten()
    bins = int(len(m) * 0.01) + 1
    plt.hist(m.numpy(), bins=bins, density=True, alpha=0.6, label="Model", color="blue")
    plt.hist(o.numpy(), bins=bins, density=True, alpha=0.6, label="OLS", color="orange")
    for t, name, color in ((m, "Model", "blue"), (o, "OLS  ", "orange")):
        avg, std = float(t.mean()), float(t.std())
        plt.axvline(avg, color=color, linestyle="--", label=f"{name} Residual Avg: {avg:.4f} (std={std:.4f})")
    plt.title(title)
    plt.grid(alpha=0.5)
    plt.legend()
    return fig


def estimation_plots(tb, model_ests: Tensor, ols_ests: Tensor, trues: Tensor, est_kind: str = "alpha") -> None:
    for stock in range(min(model_ests.shape[1], 9)):
        fig = plt.figure(figsize=FIGSIZE)
        plt.title(f"Model vs OLS {est_kind} estimation (Stock {stock})")
        x = np.arange(model_ests.shape[0])
        plt.plot(x, trues[:, stock].numpy(), color="magenta", linestyle="--", label=f"True {est_kind}", alpha=0.5)
        plt.scatter(x, model_ests[:, stock].numpy(), label="Model", marker=".", color="blue")
        plt.scatter(x, ols_ests[:, stock].numpy(), label="OLS", marker=".", color="orange")
        plt.legend()
        plt.grid(alpha=0.5)
        tb.add_figure(f"estimation/examples_{est_kind}", fig, global_step=stock)


def estimation_scatter(model_ests: Tensor, ols_ests: Tensor, trues: Tensor, est_kind: str = "alpha"):
    fig, (ax1, ax2) = plt.subplots(2, 1, figsize=FIGSIZE, sharex=True, sharey=True)
    fig.suptitle(f"Ground Truth {est_kind} vs Estimated {est_kind}")
    m, o, t = model_ests.flatten(), ols_ests.flatten(), trues.flatten()
    lims = (float(t.min()), float(t.max()))
    for ax, est, name, color in ((ax1, m, "Model", "blue"), (ax2, o, "OLS", "orange")):
        ax.set_title(f"{name} corr={_corr(est, t):.4f}")
        ax.set_ylabel(f"{name} {est_kind}")
        ax.plot(lims, lims, color="magenta", linestyle="--")
        ax.grid()
        ax.scatter(t.numpy(), est.numpy(), marker=".", alpha=0.15, color=color)
    ax2.set_xlabel(f"Ground Truth {est_kind}")
    return fig
