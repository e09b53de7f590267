"""Model registry (reference: ``get_model_class``, `train.py:45-67`).

``loss.module_class`` selects the LightningModule; ``model.arch`` (an MI355X
extension, default ``lstm``) selects the encoder family: the reference LSTM, or the
``BASELINE.json`` north-star extras ``mlp`` / ``transformer``.
"""
from __future__ import annotations

from typing import Any, Dict

from .lstm import FinancialLstm, FinancialLstmCombined, FinancialLstmMse, FinancialLstmNll, LSTMStack

_MODEL_CLASSES: Dict[str, Any] = {
    "FinancialLstmMse": FinancialLstmMse,
    "FinancialLstmNll": FinancialLstmNll,
    "FinancialLstmCombined": FinancialLstmCombined,
}


def register_model_class(name: str, cls) -> None:
    _MODEL_CLASSES[name] = cls


def get_model_class(module_class_name: str, arch: str = "lstm"):
    """Map a config string to its module class (same errors as the reference)."""
    if arch != "lstm":
        from . import extras  # noqa: F401  (registers the extra families)

        module_class_name = module_class_name.replace("FinancialLstm", extras.ARCH_PREFIX[arch])
    if module_class_name not in _MODEL_CLASSES:
        raise ValueError(f"Unknown module class: {module_class_name}. Available: {list(_MODEL_CLASSES.keys())}")
    return _MODEL_CLASSES[module_class_name]


def model_params_from_config(cfg) -> Dict[str, Any]:
    """Constructor kwargs from the composed config (`train.py:124-136`)."""
    m = cfg.model
    params = {
        "input_size": m.input_size,
        "hidden_size": m.hidden_size,
        "num_layers": m.num_layers,
        "dropout": m.dropout,
        "learning_rate": m.learning_rate,
    }
    # reference never forwards weight_decay: default 1e-5 unless the config sets it
    if "weight_decay" in m:
        params["weight_decay"] = m.weight_decay
    for k in ("num_heads", "mlp_ratio", "norm"):
        if k in m:
            params[k] = m[k]
    if m.get("arch", "lstm") == "mlp":
        params["lookback"] = int(cfg.datamodule.lookback_window)
    if cfg.loss.name == "combined":
        params["mse_weight"] = cfg.loss.mse_weight
    if "nll_mode" in cfg.loss:
        params["nll_mode"] = cfg.loss.nll_mode
    if "optimizer" in m:
        params["optimizer"] = m.optimizer
    if "backend" in m:
        params["backend"] = m.backend
    return params


__all__ = ["FinancialLstm", "FinancialLstmMse", "FinancialLstmNll", "FinancialLstmCombined", "LSTMStack",
           "get_model_class", "register_model_class", "model_params_from_config"]
