"""Public-name registry: `@export('paillier.fixedpoint.encode')` makes the object reachable as
`efl.paillier.fixedpoint.encode`, the dotted names efls-train exposes
(efls-train/python/efl/exporter.py:44-53, filled at efl/__init__.py:47)."""
from __future__ import annotations

import types

_registry: dict[str, object] = {}


def export(name: str):
    def deco(obj):
        if name in _registry and _registry[name] is not obj:
            raise ImportError(f"efl: public name {name!r} exported twice")
        _registry[name] = obj
        return obj
    return deco


def filldict(namespace: dict) -> None:
    for dotted, obj in _registry.items():
        parts = dotted.split(".")
        d = namespace
        for p in parts[:-1]:
            mod = d.get(p)
            if not isinstance(mod, types.ModuleType):
                mod = types.ModuleType(p)
                d[p] = mod
            d = mod.__dict__
        d[parts[-1]] = obj
