"""Kernel-route counters: which native kernel (or library / torch fallback)
each op dispatched to, summed over the ops modules' ``_STATS`` dicts.

``bench.py`` records the routes its timed steps take (``config.routes``) and
the GPU convergence regression records the routes its training took; the
test requires the bench's set to be a subset of the trained one, so every
kernel the headline number runs on has also been trained with (VERDICT r3
item 5)."""
from __future__ import annotations

import importlib
from typing import Dict, Iterable, List

_MODULES = ("attention", "batchnorm", "bn_fold", "conv1x1", "conv_igemm", "depthwise", "fused", "layernorm",
            "linear", "loss", "patch_embed", "pool", "stem")


def _tables():
    for name in _MODULES:
        mod = importlib.import_module(f"distributed_model_parallel_amd.ops.{name}")
        for attr in ("_STATS", "_STATS_FUSED"):
            tab = getattr(mod, attr, None)
            if isinstance(tab, dict):
                yield name, tab


def route_counts() -> Dict[str, int]:
    """{"module.route": calls} for every counter of every ops module."""
    return {f"{mod}.{k}": int(v) for mod, tab in _tables() for k, v in tab.items()}


def reset_routes() -> None:
    for _, tab in _tables():
        for k in tab:
            tab[k] = 0


def active(counts: Dict[str, int]) -> List[str]:
    return sorted(k for k, v in counts.items() if v > 0)


def diff(after: Dict[str, int], before: Dict[str, int]) -> Dict[str, int]:
    return {k: v - before.get(k, 0) for k, v in after.items() if v - before.get(k, 0) > 0}


def missing(required: Iterable[str], seen: Iterable[str]) -> List[str]:
    s = set(seen)
    return sorted(r for r in required if r not in s)
