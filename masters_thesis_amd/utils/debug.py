"""Serialize / launch-blocking debug mode (SURVEY §5 "Race detection": the MI355X counterpart of
``CUDA_LAUNCH_BLOCKING=1`` + compute-sanitizer runs of the reference's implicit CUDA stack).

``Trainer(debug_serialize=True)`` (config ``trainer.debug_serialize=true``, or ``MTA_DEBUG_SERIALIZE=1``) sets the
HIP runtime switches that make every kernel launch and copy synchronous before the process touches the GPU:

* ``AMD_SERIALIZE_KERNEL=3`` -- wait for the device to be idle before and after every kernel,
* ``AMD_SERIALIZE_COPY=3``   -- the same for every copy,
* ``HIP_LAUNCH_BLOCKING=1``  -- host-side blocking launches,

and turns captured HIP graphs off (a replayed graph would hide the launch boundaries again).  A kernel fault or a
bounded-wait give-up is then reported at the launch that caused it, not at a later synchronisation.  The switches
only act when set before the HIP runtime initialises; ``apply_serialize_env`` says so when it is too late.
"""
from __future__ import annotations

import os
from typing import Dict

SERIALIZE_ENV: Dict[str, str] = {"AMD_SERIALIZE_KERNEL": "3", "AMD_SERIALIZE_COPY": "3", "HIP_LAUNCH_BLOCKING": "1"}


def serialize_requested(flag: bool = False) -> bool:
    return bool(flag) or os.environ.get("MTA_DEBUG_SERIALIZE", "0") == "1"


def apply_serialize_env() -> bool:
    """Export the serialize switches; returns False (and warns) if the HIP runtime is already initialised."""
    for k, v in SERIALIZE_ENV.items():
        os.environ[k] = v
    try:
        import torch

        late = torch.cuda.is_available() and torch.cuda.is_initialized()
    except Exception:  # pragma: no cover
        late = False
    if late:
        print("[debug] serialize mode requested after the HIP runtime initialised: AMD_SERIALIZE_KERNEL / "
              "HIP_LAUNCH_BLOCKING take effect only in a fresh process (set MTA_DEBUG_SERIALIZE=1 at launch)",
              flush=True)
    return not late
