"""Minimal Hydra/OmegaConf-compatible config composition.

The reference composes its configs with Hydra (``isaacgymenvs/__init__.py:35-38``,
``train.py:86``) and registers four OmegaConf resolvers
(``isaacgymenvs/__init__.py:8-11``): ``eq``, ``contains``, ``if`` and
``resolve_default``.  Hydra and OmegaConf are not available in this image, so
this module restates the subset the in-scope configs use:

* the ``defaults`` list of ``cfg/config.yaml`` (``task``, ``train: ${task}PPO``);
* command-line style overrides ``group=choice`` and ``a.b.c=value``;
* absolute ``${a.b}`` and relative ``${..a}`` interpolation (one dot = the
  containing node, each further dot one level up), with nested resolver calls.

If real Hydra/OmegaConf are importable they are not required; the composed
result is a plain ``dict`` exactly like ``omegaconf_to_dict(cfg)``.
"""
from __future__ import annotations

import copy
import os
from typing import Any, Dict, List, Optional

import yaml

CFG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cfg")


def _to_bool_str(x):
    return str(x).lower()


RESOLVERS = {
    "eq": lambda x, y: _to_bool_str(x) == _to_bool_str(y),
    "contains": lambda x, y: _to_bool_str(x) in _to_bool_str(y),
    "if": lambda pred, a, b: a if pred else b,
    "resolve_default": lambda default, arg: default if arg == "" else arg,
}


def _load(path: str) -> dict:
    with open(path) as f:
        return yaml.safe_load(f) or {}


def _set_path(d: dict, dotted: str, value: Any) -> None:
    keys = dotted.split(".")
    cur = d
    for k in keys[:-1]:
        if k not in cur or not isinstance(cur[k], dict):
            cur[k] = {}
        cur = cur[k]
    cur[keys[-1]] = value


def _parse_value(s: str) -> Any:
    if s == "":
        return ""
    try:
        return yaml.safe_load(s)
    except yaml.YAMLError:
        return s


# ----------------------------------------------------------------- interpolation
class _Resolver:
    def __init__(self, root: dict):
        self.root = root
        self._busy = set()

    def lookup(self, path: List[str], ref: str) -> Any:
        """`path` is the key path of the node holding the string being resolved."""
        if ref.startswith("."):
            ndots = len(ref) - len(ref.lstrip("."))
            rest = ref[ndots:]
            base = path[:-1]  # the containing node
            base = base[: len(base) - (ndots - 1)] if ndots > 1 else base
            keys = base + ([k for k in rest.split(".") if k] if rest else [])
        else:
            keys = [k for k in ref.split(".") if k]
        node = self.root
        for k in keys:
            if isinstance(node, dict) and k in node:
                node = node[k]
            elif isinstance(node, list) and k.isdigit():
                node = node[int(k)]
            else:
                raise KeyError(f"interpolation ${{{ref}}} at {'.'.join(path)}: missing key {k}")
        return self.resolve_value(node, keys)

    def resolve_value(self, v: Any, path: List[str]) -> Any:
        if isinstance(v, str) and "${" in v:
            key = tuple(path)
            if key in self._busy:
                raise ValueError(f"interpolation cycle at {'.'.join(path)}")
            self._busy.add(key)
            try:
                return self._resolve_str(v, path)
            finally:
                self._busy.discard(key)
        return v

    def _resolve_str(self, s: str, path: List[str]) -> Any:
        out, i, parts = [], 0, []
        while i < len(s):
            j = s.find("${", i)
            if j < 0:
                parts.append(s[i:])
                break
            parts.append(s[i:j])
            k = self._match(s, j)
            parts.append(self._eval(s[j + 2:k], path))
            i = k + 1
        parts = [p for p in parts if not (isinstance(p, str) and p == "")]
        if len(parts) == 1:
            return parts[0]
        return "".join(str(p) for p in parts)

    @staticmethod
    def _match(s: str, start: int) -> int:
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
        raise ValueError(f"unbalanced interpolation: {s}")

    def _split_args(self, s: str) -> List[str]:
        args, depth, cur, quote = [], 0, "", None
        i = 0
        while i < len(s):
            c = s[i]
            if quote:
                cur += c
                if c == quote:
                    quote = None
            elif c in "\"'":
                quote = c
                cur += c
            elif s.startswith("${", i):
                depth += 1
                cur += "${"
                i += 2
                continue
            elif c == "}":
                depth -= 1
                cur += c
            elif c == "," and depth == 0:
                args.append(cur)
                cur = ""
            else:
                cur += c
            i += 1
        args.append(cur)
        return [a.strip() for a in args]

    def _eval(self, body: str, path: List[str]) -> Any:
        head = body.split(":", 1)[0]
        if ":" in body and head in RESOLVERS and not body.startswith("."):
            raw_args = self._split_args(body.split(":", 1)[1])
            args = []
            for a in raw_args:
                if "${" in a:
                    args.append(self._resolve_str(a, path))
                elif len(a) >= 2 and a[0] == a[-1] and a[0] in "\"'":
                    args.append(a[1:-1])
                else:
                    args.append(_parse_value(a))
            return RESOLVERS[head](*args)
        return self.lookup(path, body)


def resolve(cfg: dict) -> dict:
    root = copy.deepcopy(cfg)
    r = _Resolver(root)

    def walk(node, path):
        if isinstance(node, dict):
            return {k: walk(v, path + [k]) for k, v in node.items()}
        if isinstance(node, list):
            return [walk(v, path + [str(i)]) for i, v in enumerate(node)]
        return r.resolve_value(node, path)

    return walk(root, [])


# ----------------------------------------------------------------- composition
def compose(config_name: str = "config", overrides: Optional[List[str]] = None, cfg_dir: str = CFG_DIR,
            resolve_interpolations: bool = True) -> dict:
    """``hydra.compose(config_name, overrides)`` followed by ``omegaconf_to_dict``."""
    overrides = list(overrides or [])
    base = _load(os.path.join(cfg_dir, f"{config_name}.yaml"))
    defaults = base.pop("defaults", [])
    choices: Dict[str, str] = {}
    for d in defaults:
        if isinstance(d, dict):
            for k, v in d.items():
                choices[k] = v
    rest = []
    for o in overrides:
        k, _, v = o.partition("=")
        k = k.lstrip("+")
        if k in ("task", "train"):
            choices[k] = v
        else:
            rest.append((k, v))
    task_name = choices.get("task")
    train_name = str(choices.get("train", "")).replace("${task}", task_name or "")
    cfg = dict(base)
    if task_name:
        cfg["task"] = _load(os.path.join(cfg_dir, "task", f"{task_name}.yaml"))
    if train_name and os.path.exists(os.path.join(cfg_dir, "train", f"{train_name}.yaml")):
        cfg["train"] = _load(os.path.join(cfg_dir, "train", f"{train_name}.yaml"))
    for k, v in rest:
        _set_path(cfg, k, _parse_value(v))
    return resolve(cfg) if resolve_interpolations else cfg
