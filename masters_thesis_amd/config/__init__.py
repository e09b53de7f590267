"""Self-contained Hydra/OmegaConf-compatible configuration system."""
from .nodes import DictConfig, ListConfig, OmegaConf, InterpolationError, MISSING
from .composer import Override, parse_override, compose, expand_sweep, ConfigCompositionError
from .app import main, run
from .resolvers import register_default_resolvers

__all__ = [
    "DictConfig", "ListConfig", "OmegaConf", "InterpolationError", "MISSING",
    "Override", "parse_override", "compose", "expand_sweep", "ConfigCompositionError",
    "main", "run", "register_default_resolvers",
]
