"""Host-native runtime pieces (C++, pybind11): ``_omnia_native``.

Built in-tree by :mod:`omnia_amd.native.build` (also from ``__graft_entry__.build``);
imported lazily, failing loudly when missing."""
from __future__ import annotations

import importlib

_mod = None


def native():
    global _mod
    if _mod is None:
        try:
            _mod = importlib.import_module("omnia_amd.native._omnia_native")
        except ImportError:
            from .build import build

            build()
            _mod = importlib.import_module("omnia_amd.native._omnia_native")
    return _mod
