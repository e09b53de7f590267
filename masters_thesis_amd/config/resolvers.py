"""Resolvers the configs rely on.

``input_size_from_interaction`` is the reference's custom resolver
(`train.py:39-42`, used by `configs/model/*.yaml:1`): 3 input features
``[r_s, r_m, r_s*r_m]`` when ``interaction_only`` else 5 (adds squares,
`src/common.py:115-130`).
"""
from .nodes import OmegaConf


def register_default_resolvers() -> None:
    OmegaConf.register_new_resolver(
        "input_size_from_interaction", lambda interaction_only: 3 if interaction_only else 5, replace=True
    )


register_default_resolvers()
