"""Native (C++17) host runtime: KV block allocator / sequence tables, token loader, indexer.

Built in-tree into ``llmctl/native/_llmctl_native*.so`` by ``python -m llmctl.native.build``
(g++ + pybind11, no GPU needed).  ``load()`` returns the module or None; callers keep a
pure-Python implementation of the same semantics for environments without a compiler.
"""

from __future__ import annotations

import importlib
from pathlib import Path
from typing import Optional

_mod = None
_err: Optional[str] = None


def load():
    global _mod, _err
    if _mod is not None:
        return _mod
    try:
        _mod = importlib.import_module("llmctl.native._llmctl_native")
    except Exception as e:  # not built
        _err = str(e)
        _mod = None
    return _mod


def available() -> bool:
    return load() is not None


class _LoaderShim:
    pass


class loader:  # namespace used by llmctl.io.dataset
    @staticmethod
    def TokenLoader(path, itemsize, seq_len, batch, rank, world, seed, depth=4):
        m = load()
        if m is None:
            raise ImportError(_err or "native module not built")
        return m.TokenLoader(path, itemsize, seq_len, batch, rank, world, seed, depth)
