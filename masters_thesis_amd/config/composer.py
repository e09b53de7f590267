"""Hydra-compatible config composition, override grammar and multirun sweeps.

Re-implements what the reference gets from ``@hydra.main`` (`train.py:70`,
`test.py:147`): the primary ``configs/config.yaml`` defaults list (groups,
``_self_``, ``override hydra/launcher: joblib`` — `configs/config.yaml:1-7`),
group selection (``loss=nll``), dotted value overrides
(``loss.mse_weight=0.7``), ``+key``/``++key``/``~key``, comma sweeps under
``-m`` (`sweeps/*.sh`) expanded as a cartesian product in the order Hydra's
BasicSweeper uses, and the ``outputs/<date>/<time>`` / ``multirun/<date>/<time>/<n>``
run directories with ``.hydra/{config,hydra,overrides}.yaml``.
``version_base=None`` semantics: the job does *not* chdir into its run dir.
"""
from __future__ import annotations

import copy
import dataclasses
import itertools
import os
from pathlib import Path
from typing import Any, Dict, List, Optional, Sequence, Tuple

import yaml

from .nodes import DictConfig, OmegaConf, deep_merge, del_dotted, parse_scalar, set_dotted, _split_args

__all__ = [
    "Override",
    "parse_override",
    "compose",
    "expand_sweep",
    "ConfigCompositionError",
    "HYDRA_DEFAULTS",
]


class ConfigCompositionError(ValueError):
    pass


# Defaults for the ``hydra`` node (subset of Hydra 1.3's hydra/config).
HYDRA_DEFAULTS: Dict[str, Any] = {
    "run": {"dir": "outputs/${now:%Y-%m-%d}/${now:%H-%M-%S}"},
    "sweep": {"dir": "multirun/${now:%Y-%m-%d}/${now:%H-%M-%S}", "subdir": "${hydra.job.num}"},
    "launcher": {"_target_": "basic"},
    "job": {"name": "app", "chdir": False, "num": 0, "override_dirname": "", "id": "0"},
    "mode": "RUN",
    "output_subdir": ".hydra",
    "verbose": False,
}

# Built-in launcher group options (``override hydra/launcher: <name>``).
LAUNCHER_PRESETS: Dict[str, Dict[str, Any]] = {
    "basic": {"_target_": "basic"},
    "joblib": {"_target_": "joblib", "n_jobs": -1, "backend": None, "prefer": "processes", "verbose": 0,
               "max_retries": 0, "heartbeat_timeout_s": 0},
    "gpu_pool": {"_target_": "gpu_pool", "devices": None, "jobs_per_device": 1, "max_jobs_per_device": 4, "n_jobs": None, "max_retries": 0,
                 "heartbeat_timeout_s": 0},
}


@dataclasses.dataclass
class Override:
    """One CLI override: ``[+|++|~]key[@pkg]=value``."""

    key: str
    value: Any  # parsed value, or a list of parsed values for a sweep
    raw_value: Optional[str]
    kind: str  # "change" | "add" | "force_add" | "delete"
    is_sweep: bool = False

    def text(self) -> str:
        prefix = {"change": "", "add": "+", "force_add": "++", "delete": "~"}[self.kind]
        if self.raw_value is None:
            return f"{prefix}{self.key}"
        return f"{prefix}{self.key}={self.raw_value}"


def _parse_sweep_fn(v: str) -> Optional[List[Any]]:
    v = v.strip()
    if v.startswith("range(") and v.endswith(")"):
        args = [parse_scalar(a) for a in _split_args(v[6:-1])]
        if len(args) == 1:
            args = [0, args[0]]
        start, stop = args[0], args[1]
        step = args[2] if len(args) > 2 else 1
        out, x = [], start
        while (step > 0 and x < stop) or (step < 0 and x > stop):
            out.append(x)
            x += step
        return out
    if v.startswith("choice(") and v.endswith(")"):
        return [parse_scalar(a) for a in _split_args(v[7:-1])]
    return None


def parse_override(text: str) -> Override:
    t = text.strip()
    kind = "change"
    if t.startswith("++"):
        kind, t = "force_add", t[2:]
    elif t.startswith("+"):
        kind, t = "add", t[1:]
    elif t.startswith("~"):
        kind, t = "delete", t[1:]
    if "=" not in t:
        if kind == "delete":
            return Override(t, None, None, "delete")
        raise ConfigCompositionError(f"Error parsing override '{text}': missing '='")
    key, raw = t.split("=", 1)
    key = key.strip()
    sweep = _parse_sweep_fn(raw)
    if sweep is not None:
        return Override(key, sweep, raw, kind, is_sweep=True)
    parts = _split_args(raw) if raw else [""]
    if len(parts) > 1:
        return Override(key, [parse_scalar(p) for p in parts], raw, kind, is_sweep=True)
    return Override(key, parse_scalar(raw), raw, kind)


def expand_sweep(overrides: Sequence[Override]) -> List[List[Override]]:
    """Cartesian product of sweep overrides (Hydra BasicSweeper order: first key outermost)."""
    axes: List[List[Override]] = []
    for o in overrides:
        if o.is_sweep:
            raws = _split_args(o.raw_value) if _parse_sweep_fn(o.raw_value) is None else [str(v) for v in o.value]
            axes.append(
                [Override(o.key, v, r, o.kind) for v, r in zip(o.value, raws)]
            )
        else:
            axes.append([o])
    return [list(combo) for combo in itertools.product(*axes)]


# --------------------------------------------------------------------------- #
# composition
# --------------------------------------------------------------------------- #
def _load_yaml(path: Path) -> dict:
    with open(path) as f:
        data = yaml.safe_load(f)
    return data or {}


def _is_group(config_dir: Path, name: str) -> bool:
    return (config_dir / name).is_dir()


def _group_option_file(config_dir: Path, group: str, option: str) -> Path:
    p = config_dir / group / f"{option}.yaml"
    if not p.exists():
        avail = sorted(x.stem for x in (config_dir / group).glob("*.yaml")) if (config_dir / group).is_dir() else []
        raise ConfigCompositionError(
            f"Could not find '{group}/{option}'\nAvailable options in '{group}':\n\t" + "\n\t".join(avail)
        )
    return p


def compose(
    config_dir: os.PathLike,
    config_name: str = "config",
    overrides: Sequence[str | Override] = (),
    *,
    allow_sweep: bool = False,
) -> Tuple[DictConfig, DictConfig, Dict[str, Optional[str]]]:
    """Compose ``config_name`` + overrides.

    Returns ``(job_cfg, hydra_cfg, choices)`` where ``job_cfg`` excludes the
    ``hydra`` node (as Hydra passes it to the task function) and ``choices``
    maps each config group to its selected option (``hydra.runtime.choices``).
    """
    config_dir = Path(config_dir)
    ovs = [parse_override(o) if isinstance(o, str) else o for o in overrides]
    for o in ovs:
        if o.is_sweep and not allow_sweep:
            raise ConfigCompositionError(
                f"Ambiguous value for argument '{o.text()}'\n"
                "1. To use it as a list, use key=[value1,value2]\n"
                "2. To use it as string, quote the value: key=\\'value1,value2\\'\n"
                "3. To sweep over it, add --multirun to your command line"
            )

    primary = _load_yaml(config_dir / f"{config_name}.yaml")
    defaults = primary.pop("defaults", [])

    # ---- defaults list -> ordered entries ----------------------------------
    entries: List[Tuple[str, Optional[str]]] = []  # (group or "_self_", option)
    hydra_choices: Dict[str, str] = {"hydra/launcher": "basic"}
    for d in defaults:
        if d == "_self_":
            entries.append(("_self_", None))
        elif isinstance(d, str):
            grp, _, opt = d.partition("/")
            entries.append((grp, opt or None))
        elif isinstance(d, dict):
            (k, v), = d.items()
            k = str(k)
            if k.startswith("override "):
                grp = k[len("override "):].strip()
                if grp.startswith("hydra/"):
                    hydra_choices[grp] = v
                else:
                    entries = [(g, v if g == grp else o) for g, o in entries]
                continue
            if k.startswith("optional "):
                k = k[len("optional "):].strip()
            if k.startswith("hydra/"):
                hydra_choices[k] = v
                continue
            entries.append((k, v))
    if ("_self_", None) not in entries:
        entries.append(("_self_", None))

    # ---- group overrides from the CLI --------------------------------------
    group_names = {g for g, _ in entries if g != "_self_"}
    value_overrides: List[Override] = []
    for o in ovs:
        if o.key.startswith("hydra/"):
            hydra_choices[o.key] = o.value
            continue
        if o.key.startswith("hydra."):
            value_overrides.append(o)
            continue
        if _is_group(config_dir, o.key) and "." not in o.key:
            if o.kind == "delete":
                entries = [(g, v) for g, v in entries if g != o.key]
                group_names.discard(o.key)
            elif o.key in group_names:
                if o.kind == "add":
                    raise ConfigCompositionError(
                        f"Could not append to config. An item is already at '{o.key}'."
                    )
                entries = [(g, o.value if g == o.key else v) for g, v in entries]
            else:
                if o.kind == "change":
                    raise ConfigCompositionError(
                        f"Could not override '{o.key}'. No match in the defaults list.\n"
                        f"To append to your default list use +{o.key}={o.raw_value}"
                    )
                # appended groups go before _self_ like Hydra's defaults tree
                idx = [g for g, _ in entries].index("_self_")
                entries.insert(idx, (o.key, o.value))
                group_names.add(o.key)
        else:
            value_overrides.append(o)

    # ---- merge --------------------------------------------------------------
    content: dict = {}
    choices: Dict[str, Optional[str]] = {}
    for grp, opt in entries:
        if grp == "_self_":
            deep_merge(content, copy.deepcopy(primary))
            continue
        choices[grp] = opt
        if opt is None:
            continue
        node = _load_yaml(_group_option_file(config_dir, grp, str(opt)))
        sub: dict = content
        for p in grp.split("/")[:-1]:
            sub = sub.setdefault(p, {})
        leaf = grp.split("/")[-1]
        if isinstance(sub.get(leaf), dict):
            deep_merge(sub[leaf], node)
        else:
            sub[leaf] = node

    # ---- hydra node ---------------------------------------------------------
    hydra_node = copy.deepcopy(HYDRA_DEFAULTS)
    launcher_name = str(hydra_choices.get("hydra/launcher", "basic"))
    if launcher_name not in LAUNCHER_PRESETS:
        raise ConfigCompositionError(
            f"Could not find 'hydra/launcher/{launcher_name}'. Available: {sorted(LAUNCHER_PRESETS)}"
        )
    hydra_node["launcher"] = copy.deepcopy(LAUNCHER_PRESETS[launcher_name])
    if "hydra" in content:
        deep_merge(hydra_node, content.pop("hydra"))
    content["hydra"] = hydra_node

    # ---- value overrides ------------------------------------------------------
    for o in value_overrides:
        if o.kind == "delete":
            del_dotted(content, o.key)
        elif o.kind == "add":
            _check_absent(content, o.key)
            set_dotted(content, o.key, o.value)
        elif o.kind == "force_add":
            set_dotted(content, o.key, o.value)
        else:
            set_dotted(content, o.key, o.value, must_exist=True)

    full = DictConfig(content)
    hydra_cfg = full["hydra"]
    hydra_cfg["runtime"] = {
        "choices": {**{k: v for k, v in choices.items()}, **hydra_choices},
        "config_name": config_name,
        "config_sources": [str(config_dir)],
    }
    hydra_cfg["overrides"] = {"task": [o.text() for o in ovs if not o.key.startswith("hydra")]}
    # the task function sees the config WITHOUT the hydra node (as with @hydra.main);
    # ``${hydra:key}`` stays resolvable through a resolver bound to this run's hydra node
    job_cfg = DictConfig({k: v for k, v in full._content.items() if k != "hydra"})
    hydra_view = full["hydra"]
    OmegaConf.register_new_resolver("hydra", lambda key, _h=hydra_view: _h._select("hydra." + str(key)), replace=True)
    return job_cfg, hydra_view, choices


def _check_absent(content: dict, dotted: str) -> None:
    node = content
    parts = dotted.split(".")
    for p in parts[:-1]:
        if p not in node:
            return
        node = node[p]
    if isinstance(node, dict) and parts[-1] in node:
        raise ConfigCompositionError(
            f"Could not append to config. An item is already at '{dotted}'."
        )


def override_dirname(overrides: Sequence[Override], exclude: Sequence[str] = ()) -> str:
    items = sorted(o.text() for o in overrides if o.key not in exclude and not o.key.startswith("hydra"))
    return ",".join(items)
