"""Plugin registry for the entry-point groups the reference declares (``pyproject.toml:77-81``:
``llmctl.plugins.{kernels,quantizers,exporters,schedulers}:register`` — modules that did
not exist there).  Built-ins register themselves; third-party packages add entries under
the ``llmctl.plugins`` entry-point group (each entry point is a ``register(registry)``
callable).
"""

from __future__ import annotations

from typing import Any, Callable, Dict

GROUPS = ("kernels", "quantizers", "exporters", "schedulers")


class Registry:
    def __init__(self):
        self._items: Dict[str, Dict[str, Any]] = {g: {} for g in GROUPS}
        self._loaded = False

    def add(self, group: str, name: str, obj: Any) -> None:
        if group not in self._items:
            raise KeyError(f"unknown plugin group {group}")
        self._items[group][name] = obj

    def get(self, group: str, name: str) -> Any:
        self.load()
        try:
            return self._items[group][name]
        except KeyError:
            raise KeyError(f"no {group} plugin named {name!r} (have {sorted(self._items[group])})") from None

    def names(self, group: str):
        self.load()
        return sorted(self._items[group])

    def load(self) -> None:
        if self._loaded:
            return
        self._loaded = True
        from . import exporters, kernels, quantizers, schedulers

        for mod in (kernels, quantizers, exporters, schedulers):
            mod.register(self)
        try:
            from importlib.metadata import entry_points

            eps = entry_points()
            group = eps.select(group="llmctl.plugins") if hasattr(eps, "select") else eps.get("llmctl.plugins", [])
            for ep in group:
                if ep.value.startswith("llmctl.plugins."):
                    continue  # built-ins already registered
                try:
                    ep.load()(self)
                except Exception:
                    pass
        except Exception:
            pass


registry = Registry()
