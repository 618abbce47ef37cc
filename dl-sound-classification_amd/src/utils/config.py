"""Minimal Hydra/OmegaConf-compatible config composition and ``_target_`` instantiation.

hydra-core 1.3.2 / omegaconf 2.3.0 (reference uv.lock:733,1326) are not installed in this image, so
``scripts/train.py`` composes the same YAML tree (configs/training.yaml defaults list:
base_training + dataset/<name> + model/<name> + _self_) with the same override grammar
(``key.sub=value``, ``+key=value``, ``group=option``) and ``${a.b}`` interpolation.  When hydra is
importable the real one can be used instead; the semantics the reference relies on are the same.
"""
from __future__ import annotations

import copy
import importlib
import re
from pathlib import Path
from typing import Any

import yaml


class Cfg(dict):
    """dict with attribute access and ``get`` on dotted paths (the subset of DictConfig in use)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    @staticmethod
    def wrap(x):
        if isinstance(x, dict) and not isinstance(x, Cfg):
            return Cfg({k: Cfg.wrap(v) for k, v in x.items()})
        if isinstance(x, list):
            return [Cfg.wrap(v) for v in x]
        return x


def to_container(x):
    if isinstance(x, dict):
        return {k: to_container(v) for k, v in x.items()}
    if isinstance(x, list):
        return [to_container(v) for v in x]
    return x


def _merge(a: dict, b: dict) -> dict:
    out = copy.deepcopy(a)
    for k, v in b.items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = _merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


class _Loader(yaml.SafeLoader):
    """SafeLoader that also reads ``1e-4``-style floats as floats (as OmegaConf's loader does)."""


_Loader.add_implicit_resolver(
    "tag:yaml.org,2002:float",
    re.compile(r"""^(?:[-+]?(?:[0-9][0-9_]*)\.[0-9_]*(?:[eE][-+]?[0-9]+)?
    |[-+]?(?:[0-9][0-9_]*)(?:[eE][-+]?[0-9]+)
    |\.[0-9_]+(?:[eE][-+][0-9]+)?
    |[-+]?\.(?:inf|Inf|INF)
    |\.(?:nan|NaN|NAN))$""", re.X), list("-+0123456789."))


def _load_yaml(path: Path) -> dict:
    with open(path) as f:
        return yaml.load(f, Loader=_Loader) or {}


def _compose(cfg_dir: Path, name: str, group_choices: dict) -> dict:
    raw = _load_yaml(cfg_dir / f"{name}.yaml")
    defaults = raw.pop("defaults", [])
    out: dict = {}
    self_done = False
    for d in defaults:
        if d == "_self_":
            out = _merge(out, raw)
            self_done = True
            continue
        if isinstance(d, str):
            out = _merge(out, _compose(cfg_dir, d, group_choices))
            continue
        (group, choice), = d.items()
        if group.startswith("override "):
            continue  # hydra/* logging overrides have no effect here
        choice = group_choices.get(group, choice)
        sub = _load_yaml(cfg_dir / group / f"{choice}.yaml")
        sub.pop("defaults", None)
        out = _merge(out, {group: sub})
    if not self_done:
        out = _merge(out, raw)
    return out


def _parse_value(s: str):
    try:
        return yaml.load(s, Loader=_Loader)
    except yaml.YAMLError:
        return s


def _set_path(d: dict, path: str, value, create: bool):
    keys = path.split(".")
    cur = d
    for k in keys[:-1]:
        if k not in cur or not isinstance(cur[k], dict):
            if not create and k not in cur:
                raise KeyError(f"override key '{path}' not in config (use +{path}=...)")
            cur[k] = {}
        cur = cur[k]
    if keys[-1] not in cur and not create:
        raise KeyError(f"override key '{path}' not in config (use +{path}=...)")
    cur[keys[-1]] = value


_INTERP = re.compile(r"\$\{([^}]+)\}")


def _resolve(node, root):
    if isinstance(node, dict):
        return {k: _resolve(v, root) for k, v in node.items()}
    if isinstance(node, list):
        return [_resolve(v, root) for v in node]
    if isinstance(node, str):
        m = _INTERP.fullmatch(node.strip())
        if m:
            return _resolve(_lookup(root, m.group(1)), root)
        return _INTERP.sub(lambda mm: str(_resolve(_lookup(root, mm.group(1)), root)), node)
    return node


def _lookup(root, path):
    if path.startswith("now:"):
        import datetime
        return datetime.datetime.now().strftime(path[4:])
    cur = root
    for k in path.split("."):
        cur = cur[k]
    return cur


def compose(config_dir: str | Path, config_name: str, overrides: list[str] | None = None) -> Cfg:
    cfg_dir = Path(config_dir)
    overrides = list(overrides or [])
    groups = {p.name for p in cfg_dir.iterdir() if p.is_dir()}
    choices, values = {}, []
    for ov in overrides:
        key, _, val = ov.partition("=")
        if key.lstrip("+") in groups and "." not in key:
            choices[key.lstrip("+")] = val
        else:
            values.append((key, val))
    cfg = _compose(cfg_dir, config_name, choices)
    for key, val in values:
        create = key.startswith("+")
        _set_path(cfg, key.lstrip("+"), _parse_value(val), create)
    return Cfg.wrap(_resolve(cfg, cfg))


def locate(path: str):
    mod, _, name = path.rpartition(".")
    try:
        return getattr(importlib.import_module(mod), name)
    except (ImportError, AttributeError):
        parent, _, attr = mod.rpartition(".")
        return getattr(getattr(importlib.import_module(parent), attr), name)


def instantiate(cfg: Any, **kwargs):
    """hydra.utils.instantiate for the subset in use: ``_target_`` + kwargs (recursive)."""
    if isinstance(cfg, dict) and "_target_" in cfg:
        cls = locate(cfg["_target_"])
        args = {k: instantiate(v) for k, v in cfg.items() if k not in ("_target_", "_recursive_", "_partial_")}
        args.update(kwargs)
        return cls(**args)
    if isinstance(cfg, dict):
        return Cfg({k: instantiate(v) for k, v in cfg.items()})
    if isinstance(cfg, list):
        return [instantiate(v) for v in cfg]
    return cfg
