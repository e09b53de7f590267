"""OmegaConf-compatible config containers with lazy interpolation.

The reference drives everything through OmegaConf ``DictConfig`` objects
(`train.py:70-220`, `configs/config.yaml:9-13`): attribute access, ``in``
checks (`train.py:179-180`), ``${a.b}`` interpolation (`configs/config.yaml:11-12`),
custom resolvers (`train.py:39-42`, `configs/model/*.yaml:1`) and
``OmegaConf.to_container(cfg, resolve=True)`` (`train.py:201`).  OmegaConf is not
installed on the MI355X image, so this module re-implements the subset the
framework needs.  Values are stored raw and resolved on *access* against the
root, exactly like OmegaConf, so a CLI override of ``model.learning_rate``
changes ``logger.version`` too.
"""
from __future__ import annotations

import copy
import os
import re
from typing import Any, Callable, Dict, Iterator, List, Optional

import yaml

__all__ = ["DictConfig", "ListConfig", "OmegaConf", "InterpolationError", "MISSING"]

MISSING = "???"


class InterpolationError(KeyError):
    pass


_RESOLVERS: Dict[str, Callable[..., Any]] = {}


def _oc_env(name, default=None):
    return os.environ.get(str(name), default)


def _oc_select(key, default=None, *, _root=None):
    try:
        return _root._select(str(key))
    except (KeyError, InterpolationError):
        return default


_RESOLVERS["oc.env"] = _oc_env
_RESOLVERS["oc.select"] = _oc_select


def _now(fmt="%Y-%m-%d_%H-%M-%S"):
    import datetime

    return datetime.datetime.now().strftime(str(fmt))


_RESOLVERS["now"] = _now


# --------------------------------------------------------------------------- #
# interpolation parsing
# --------------------------------------------------------------------------- #
def _find_close(s: str, start: int) -> int:
    """Index of the ``}`` that closes the ``${`` starting at ``start``."""
    depth = 0
    i = start
    while i < len(s):
        if s.startswith("${", i):
            depth += 1
            i += 2
            continue
        if s[i] == "}":
            depth -= 1
            if depth == 0:
                return i
        i += 1
    raise InterpolationError(f"unterminated interpolation in {s!r}")


def _split_args(s: str) -> List[str]:
    """Split resolver args on top-level commas (respecting ``${}``, quotes, brackets)."""
    out, cur, depth, quote = [], [], 0, None
    i = 0
    while i < len(s):
        c = s[i]
        if quote:
            cur.append(c)
            if c == quote:
                quote = None
        elif c in "'\"":
            quote = c
            cur.append(c)
        elif s.startswith("${", i):
            depth += 1
            cur.append("${")
            i += 2
            continue
        elif c in "[{(":
            depth += 1
            cur.append(c)
        elif c in "]})":
            depth -= 1
            cur.append(c)
        elif c == "," and depth == 0:
            out.append("".join(cur).strip())
            cur = []
        else:
            cur.append(c)
        i += 1
    if cur or out:
        out.append("".join(cur).strip())
    return out


def parse_scalar(text: str) -> Any:
    """YAML-1.1-ish scalar parsing, as OmegaConf/Hydra do for override values."""
    t = text.strip()
    if t == "":
        return ""
    if (t[0] == t[-1]) and t[0] in "'\"" and len(t) >= 2:
        return t[1:-1]
    low = t.lower()
    if low in ("null", "~", "none"):
        return None
    if low == "true":
        return True
    if low == "false":
        return False
    try:
        if re.fullmatch(r"[-+]?\d+", t):
            return int(t)
        if re.fullmatch(r"[-+]?(\d+\.\d*|\.\d+|\d+)([eE][-+]?\d+)?", t) or re.fullmatch(
            r"[-+]?(inf|nan)", low
        ):
            return float(t)
    except ValueError:
        pass
    if t.startswith("[") or t.startswith("{"):
        try:
            return yaml.safe_load(t)
        except yaml.YAMLError:
            return t
    return t


# --------------------------------------------------------------------------- #
# containers
# --------------------------------------------------------------------------- #
class _Node:
    __slots__ = ()


def _wrap(value, root, path):
    if isinstance(value, dict):
        return DictConfig(value, _root=root, _path=path)
    if isinstance(value, list):
        return ListConfig(value, _root=root, _path=path)
    return value


class DictConfig(_Node):
    """Dict-backed config node.  ``_content`` holds raw (unresolved) values."""

    def __init__(self, content: Optional[dict] = None, *, _root: "DictConfig" = None, _path: str = ""):
        object.__setattr__(self, "_content", {} if content is None else content)
        object.__setattr__(self, "_root", _root if _root is not None else self)
        object.__setattr__(self, "_path", _path)

    # ---- raw / resolution -------------------------------------------------
    def _child_path(self, key) -> str:
        return f"{self._path}.{key}" if self._path else str(key)

    def _resolve_value(self, raw, path):
        return self._root._resolve(raw, path)

    def _select(self, dotted: str):
        node: Any = self._root
        if dotted == "":
            return node
        for part in dotted.split("."):
            if isinstance(node, DictConfig):
                if part not in node._content:
                    raise InterpolationError(f"key '{dotted}' not found")
                node = node[part]
            elif isinstance(node, ListConfig):
                node = node[int(part)]
            else:
                raise InterpolationError(f"cannot select '{dotted}'")
        return node

    def _resolve(self, raw, path: str = "", _depth: int = 0):
        if _depth > 32:
            raise InterpolationError(f"interpolation cycle at {path}")
        if not isinstance(raw, str) or "${" not in raw:
            return raw
        s = raw
        # whole-value interpolation keeps the type
        if s.startswith("${") and _find_close(s, 0) == len(s) - 1:
            return self._resolve_one(s[2:-1], path, _depth)
        out, i = [], 0
        while i < len(s):
            j = s.find("${", i)
            if j < 0:
                out.append(s[i:])
                break
            out.append(s[i:j])
            k = _find_close(s, j)
            v = self._resolve_one(s[j + 2 : k], path, _depth)
            out.append(_to_str(v))
            i = k + 1
        return "".join(out)

    def _resolve_one(self, body: str, path: str, _depth: int):
        body = body.strip()
        m = re.match(r"^([A-Za-z_][\w.]*)\s*:(.*)$", body, re.S)
        if m:
            name, argstr = m.group(1), m.group(2)
            if name not in _RESOLVERS:
                raise InterpolationError(f"unsupported resolver '{name}' in '${{{body}}}'")
            args = [self._resolve_arg(a, path, _depth) for a in _split_args(argstr)] if argstr.strip() else []
            fn = _RESOLVERS[name]
            if fn is _oc_select:
                return fn(*args, _root=self)
            return fn(*args)
        # node reference (absolute, or relative with leading dots)
        if body.startswith("."):
            parent = path.split(".")[:-1]
            lead = len(body) - len(body.lstrip("."))
            parent = parent[: len(parent) - (lead - 1)] if lead > 1 else parent
            target = ".".join(parent + [body.lstrip(".")])
        else:
            target = body
        node = self._select_raw(target)
        if isinstance(node, (dict, list)):
            return _wrap(node, self._root, target)
        return self._resolve(node, target, _depth + 1)

    def _resolve_arg(self, a: str, path, _depth):
        if "${" in a:
            return self._resolve(a, path, _depth + 1)
        return parse_scalar(a)

    def _select_raw(self, dotted: str):
        node: Any = self._root._content
        for part in dotted.split("."):
            if isinstance(node, dict):
                if part not in node:
                    raise InterpolationError(f"interpolation key '{dotted}' not found")
                node = node[part]
            elif isinstance(node, list):
                node = node[int(part)]
            else:
                raise InterpolationError(f"interpolation key '{dotted}' not found")
        return node

    # ---- mapping protocol --------------------------------------------------
    def __getattr__(self, key):
        if key.startswith("__"):
            raise AttributeError(key)
        content = object.__getattribute__(self, "_content")
        if key not in content:
            raise AttributeError(f"Key '{key}' is not in struct ({self._path or '<root>'})")
        return self[key]

    def __setattr__(self, key, value):
        self[key] = value

    def __delattr__(self, key):
        del self._content[key]

    def __getitem__(self, key):
        raw = self._content[key]
        path = self._child_path(key)
        if isinstance(raw, (dict, list)):
            return _wrap(raw, self._root, path)
        return self._resolve_value(raw, path)

    def __setitem__(self, key, value):
        if isinstance(value, (DictConfig, ListConfig)):
            value = copy.deepcopy(value._content)
        self._content[key] = value

    def __delitem__(self, key):
        del self._content[key]

    def __contains__(self, key):
        return key in self._content

    def __iter__(self) -> Iterator[str]:
        return iter(self._content)

    def __len__(self):
        return len(self._content)

    def keys(self):
        return self._content.keys()

    def items(self):
        return [(k, self[k]) for k in self._content]

    def values(self):
        return [self[k] for k in self._content]

    def get(self, key, default=None):
        if key not in self._content:
            return default
        v = self[key]
        return default if v is None and default is not None else v

    def pop(self, key, default=None):
        if key in self._content:
            v = self[key]
            del self._content[key]
            return v
        return default

    def __eq__(self, other):
        if isinstance(other, DictConfig):
            return OmegaConf.to_container(self, resolve=True) == OmegaConf.to_container(other, resolve=True)
        if isinstance(other, dict):
            return OmegaConf.to_container(self, resolve=True) == other
        return NotImplemented

    def __repr__(self):
        return repr(self._content)

    def __deepcopy__(self, memo):
        return DictConfig(copy.deepcopy(self._content, memo))

    def __getstate__(self):
        return {"content": OmegaConf.to_container(self, resolve=False)}

    def __setstate__(self, state):
        object.__setattr__(self, "_content", state["content"])
        object.__setattr__(self, "_root", self)
        object.__setattr__(self, "_path", "")


class ListConfig(_Node):
    def __init__(self, content: list, *, _root: DictConfig, _path: str):
        self._content = content
        self._root = _root
        self._path = _path

    def __getitem__(self, i):
        raw = self._content[i]
        path = f"{self._path}.{i}"
        if isinstance(raw, (dict, list)):
            return _wrap(raw, self._root, path)
        return self._root._resolve(raw, path)

    def __setitem__(self, i, v):
        self._content[i] = v

    def __len__(self):
        return len(self._content)

    def __iter__(self):
        return (self[i] for i in range(len(self._content)))

    def __repr__(self):
        return repr(self._content)

    def __eq__(self, other):
        return list(self) == list(other)


def _to_str(v) -> str:
    if isinstance(v, (DictConfig, ListConfig)):
        return str(OmegaConf.to_container(v, resolve=True))
    if v is None:
        return "None"
    return str(v)


# --------------------------------------------------------------------------- #
# OmegaConf-style facade
# --------------------------------------------------------------------------- #
class OmegaConf:
    @staticmethod
    def register_new_resolver(name: str, fn: Callable[..., Any], replace: bool = False) -> None:
        if name in _RESOLVERS and not replace and _RESOLVERS[name] is not fn:
            raise ValueError(f"resolver '{name}' is already registered")
        _RESOLVERS[name] = fn

    @staticmethod
    def has_resolver(name: str) -> bool:
        return name in _RESOLVERS

    @staticmethod
    def clear_resolver(name: str) -> bool:
        return _RESOLVERS.pop(name, None) is not None

    @staticmethod
    def create(obj=None) -> DictConfig:
        if obj is None:
            obj = {}
        if isinstance(obj, str):
            obj = yaml.safe_load(obj) or {}
        if isinstance(obj, DictConfig):
            obj = OmegaConf.to_container(obj, resolve=False)
        return DictConfig(copy.deepcopy(obj))

    @staticmethod
    def load(path) -> DictConfig:
        with open(path) as f:
            return DictConfig(yaml.safe_load(f) or {})

    @staticmethod
    def to_container(cfg, resolve: bool = False):
        if isinstance(cfg, DictConfig):
            return {k: OmegaConf._conv(cfg, k, resolve) for k in cfg._content}
        if isinstance(cfg, ListConfig):
            return [OmegaConf._conv_list(cfg, i, resolve) for i in range(len(cfg))]
        return cfg

    @staticmethod
    def _conv(cfg: DictConfig, k, resolve):
        raw = cfg._content[k]
        if isinstance(raw, (dict, list)):
            return OmegaConf.to_container(cfg[k], resolve)
        return cfg[k] if resolve else copy.deepcopy(raw)

    @staticmethod
    def _conv_list(cfg: ListConfig, i, resolve):
        raw = cfg._content[i]
        if isinstance(raw, (dict, list)):
            return OmegaConf.to_container(cfg[i], resolve)
        return cfg[i] if resolve else copy.deepcopy(raw)

    @staticmethod
    def to_yaml(cfg, resolve: bool = False) -> str:
        return yaml.safe_dump(OmegaConf.to_container(cfg, resolve=resolve), sort_keys=False, default_flow_style=False)

    @staticmethod
    def save(cfg, path, resolve: bool = False) -> None:
        with open(path, "w") as f:
            f.write(OmegaConf.to_yaml(cfg, resolve=resolve))

    @staticmethod
    def merge(*cfgs) -> DictConfig:
        out: dict = {}
        for c in cfgs:
            src = OmegaConf.to_container(c, resolve=False) if isinstance(c, DictConfig) else copy.deepcopy(c)
            deep_merge(out, src)
        return DictConfig(out)

    @staticmethod
    def select(cfg: DictConfig, key: str, default=None):
        try:
            return cfg._select(key)
        except (KeyError, InterpolationError, IndexError, ValueError):
            return default

    @staticmethod
    def update(cfg: DictConfig, key: str, value, force_add: bool = True) -> None:
        set_dotted(cfg._root._content, key, value, force_add=force_add)


def deep_merge(dst: dict, src: dict) -> dict:
    for k, v in src.items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            deep_merge(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)
    return dst


def set_dotted(content: dict, dotted: str, value, force_add: bool = True, must_exist: bool = False) -> None:
    parts = dotted.split(".")
    node = content
    for p in parts[:-1]:
        if p not in node or not isinstance(node[p], dict):
            if must_exist:
                raise KeyError(f"Could not override '{dotted}': key '{p}' is not in the config")
            node[p] = {}
        node = node[p]
    if must_exist and parts[-1] not in node:
        raise KeyError(
            f"Could not override '{dotted}'. To append to your config use +{dotted}=..."
        )
    node[parts[-1]] = value


def del_dotted(content: dict, dotted: str) -> None:
    parts = dotted.split(".")
    node = content
    for p in parts[:-1]:
        node = node[p]
    if parts[-1] not in node:
        raise KeyError(f"Could not delete '{dotted}': key not found")
    del node[parts[-1]]
