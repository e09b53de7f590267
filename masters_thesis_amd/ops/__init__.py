"""MI355X compute ops: HIP kernels (gfx950) with pure-PyTorch CPU implementations.

Ops dispatch on the device of their inputs: GPU tensors run the hand-written
CDNA4 kernels from ``csrc/`` (``masters_thesis_amd._C``); CPU tensors run the
PyTorch reference math (used for ``BASELINE.json`` config 1 and as test oracles).
"""
from ._lib import lib, use_hip, hip_ready  # noqa: F401
