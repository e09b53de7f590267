"""Loader for the in-tree HIP extension ``masters_thesis_amd._C`` (gfx950).

On a machine with a GPU the HIP path is mandatory: if the extension is missing the
ops raise instead of silently falling back to eager PyTorch (set
``MTA_ALLOW_TORCH_FALLBACK=1`` to opt into the slow reference path explicitly).
On CPU-only machines (CI, ``BASELINE.json`` config 1) the pure-PyTorch
implementations are used.
"""
from __future__ import annotations

import os

import torch

_LIB = None
_ERR = None


def lib(required: bool = True):
    global _LIB, _ERR
    if _LIB is None and _ERR is None:
        try:
            from .. import _C  # noqa: F401

            _LIB = _C
        except ImportError as e:  # pragma: no cover - depends on build state
            _ERR = e
    if _LIB is None and required:
        raise RuntimeError(
            "masters_thesis_amd._C (HIP kernels for gfx950) is not built/importable: "
            f"{_ERR}. Run `python -m masters_thesis_amd.ops.build` (or __graft_entry__.build())."
        )
    return _LIB


def fallback_allowed() -> bool:
    return os.environ.get("MTA_ALLOW_TORCH_FALLBACK", "0") == "1"


def use_hip(t: torch.Tensor) -> bool:
    """True when ``t`` lives on the GPU and the HIP kernels must be used for it."""
    if not t.is_cuda:
        return False
    if lib(required=False) is None:
        if fallback_allowed():
            return False
        lib(required=True)  # raises loudly
    return True


def hip_ready() -> bool:
    return torch.cuda.is_available() and lib(required=False) is not None
