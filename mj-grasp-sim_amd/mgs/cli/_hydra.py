"""Hydra-compatible command-line configuration for the mgs.cli entry points.

Hydra/omegaconf are not part of this build, so this module
restates the part of Hydra the reference's CLIs use (mgs/cli/*.py,
`@hydra.main(config_path="config", config_name=...)`):

  * `config/<name>.yaml` with a `defaults:` list (`_self_`, `group: option`),
    each group option loaded from `config/<group>/<option>.yaml`;
  * command-line overrides `key=value` (`id=3`, `num_grasps=64`) and group
    selection `group=option` (`gripper=panda`), values parsed as YAML;
  * attribute access on the result (`cfg.gripper.name`).

    @main("filter_to_stable")
    def run(cfg): ...
"""
from __future__ import annotations

import functools
import os
import sys
from typing import Callable, List, Optional

import yaml

CONFIG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "config")


class Cfg(dict):
    """dict with attribute access (omegaconf DictConfig stand-in)."""

    def __getattr__(self, k):
        try:
            v = self[k]
        except KeyError as e:
            raise AttributeError(k) from e
        return Cfg(v) if isinstance(v, dict) and not isinstance(v, Cfg) else v

    def __setattr__(self, k, v):
        self[k] = v

    def get(self, k, default=None):
        v = super().get(k, default)
        return Cfg(v) if isinstance(v, dict) and not isinstance(v, Cfg) else v


def _load(path):
    with open(path) as f:
        return yaml.safe_load(f) or {}


def compose(config_name: str, overrides: Optional[List[str]] = None, config_dir: str = CONFIG_DIR) -> Cfg:
    raw = _load(os.path.join(config_dir, config_name + ".yaml"))
    defaults = raw.pop("defaults", [])
    groups = {}
    for d in defaults:
        if isinstance(d, dict):
            groups.update(d)
    plain = []
    for ov in overrides or []:
        if "=" not in ov:
            raise ValueError(f"override {ov!r} is not key=value")
        k, v = ov.split("=", 1)
        k = k.lstrip("+")
        if k in groups:
            groups[k] = v
        else:
            plain.append((k, yaml.safe_load(v)))
    cfg = Cfg(raw)
    for g, opt in groups.items():
        p = os.path.join(config_dir, g, f"{opt}.yaml")
        if not os.path.isfile(p):
            raise ValueError(f"no config {g}/{opt}.yaml")
        cfg[g] = _load(p)
    for k, v in plain:
        node = cfg
        parts = k.split(".")
        for q in parts[:-1]:
            node = node.setdefault(q, {})
        node[parts[-1]] = v
    _resolve(cfg, cfg)
    return cfg


def _resolve(node, root):
    """`${key}` / `${a.b}` interpolation of whole string values (omegaconf's
    basic form); unknown keys are left as written."""
    for k, v in list(node.items()):
        if isinstance(v, dict):
            _resolve(v, root)
        elif isinstance(v, str) and v.startswith("${") and v.endswith("}"):
            ref = root
            for q in v[2:-1].split("."):
                if not isinstance(ref, dict) or q not in ref:
                    break
                ref = ref[q]
            else:
                node[k] = ref


def main(config_name: str) -> Callable:
    """decorator: `python -m mgs.cli.<tool> key=value ...` -> fn(cfg)."""
    def deco(fn):
        @functools.wraps(fn)
        def wrapper(argv=None):
            args = sys.argv[1:] if argv is None else list(argv)
            return fn(compose(config_name, args))
        return wrapper
    return deco
