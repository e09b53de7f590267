"""Lightning-compatible checkpoint (de)serialisation.

Dict layout of a Lightning 2.x ``.ckpt`` (what `test.py:177-178` consumes through
``load_from_checkpoint``): ``epoch``, ``global_step``, ``pytorch-lightning_version``,
``state_dict`` (keys ``lstm.weight_ih_l{k}`` ... ``beta_head.bias``), ``loops``,
``callbacks``, ``optimizer_states``, ``lr_schedulers``, ``hparams_name``,
``hyper_parameters``.  MI355X additions: ``rng_states`` and ``mta`` (framework
version, world size) so ``resume=<ckpt>`` restores the full training state.
Writes are atomic (tmp file + rename) and done by global rank 0 only.
Loads use ``weights_only=True``: a checkpoint never executes code.
"""
from __future__ import annotations

import os
import random
from pathlib import Path
from typing import Any, Dict

import numpy as np
import torch

LIGHTNING_COMPAT_VERSION = "2.5.0"


def atomic_save(obj: Dict[str, Any], path: os.PathLike) -> None:
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    tmp = path.with_name(f".{path.name}.tmp{os.getpid()}")
    torch.save(obj, tmp)
    os.replace(tmp, path)


def load_checkpoint(path: os.PathLike, map_location=None) -> Dict[str, Any]:
    return torch.load(path, map_location=map_location, weights_only=True)


def capture_rng_states() -> Dict[str, Any]:
    py = random.getstate()
    npk, npst, nppos, nphas, npg = np.random.get_state()
    st = {"torch": torch.random.get_rng_state(), "python_state": list(py[1]),
          "numpy_state": npst.tolist(), "numpy_pos": int(nppos), "numpy_has_gauss": int(nphas),
          "numpy_gauss": float(npg)}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        st["cuda"] = torch.cuda.get_rng_state()
    return st


def restore_rng_states(st: Dict[str, Any]) -> None:
    if "torch" in st:
        torch.random.set_rng_state(st["torch"])
    if "cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state(st["cuda"])
    if "python_state" in st:
        random.setstate((3, tuple(st["python_state"]), None))
    if "numpy_state" in st:
        # the whole generator state (key, position, cached Gaussian): the stream continues exactly
        np.random.set_state(("MT19937", np.array(st["numpy_state"], dtype=np.uint32), int(st.get("numpy_pos", 624)),
                             int(st.get("numpy_has_gauss", 0)), float(st.get("numpy_gauss", 0.0))))
