"""MultiRLModule (reference role: rllib/core/rl_module/multi_rl_module.py).

A container of independent RLModules keyed by module (policy) id. Forward
calls take and return dicts keyed by module id; state is a dict of per-module
states, so single modules can be added, removed or restored independently.
``MultiRLModuleSpec`` records one ``RLModuleSpec`` per module; modules without
an explicit spec use the algorithm's default module class and model config,
and every module gets the spaces of the (first) agent mapped to it.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Callable, Dict, Iterable, Optional

import torch.nn as nn

from .rl_module import RLModule, RLModuleSpec

DEFAULT_MODULE_ID = "default_policy"


class MultiRLModule(nn.Module):
    def __init__(self, modules: Optional[Dict[str, RLModule]] = None):
        super().__init__()
        self._rl_modules = nn.ModuleDict(dict(modules or {}))

    # container API -----------------------------------------------------------
    def add_module(self, module_id: str, module: RLModule, *, override: bool = False):  # type: ignore[override]
        if module_id in self._rl_modules and not override:
            raise ValueError(f"module {module_id!r} exists (pass override=True)")
        self._rl_modules[module_id] = module

    def remove_module(self, module_id: str, *, raise_err_if_not_found: bool = True):
        if module_id not in self._rl_modules:
            if raise_err_if_not_found:
                raise KeyError(module_id)
            return
        del self._rl_modules[module_id]

    def keys(self):
        return list(self._rl_modules.keys())

    def items(self):
        return list(self._rl_modules.items())

    def __getitem__(self, module_id: str) -> RLModule:
        return self._rl_modules[module_id]

    def __contains__(self, module_id) -> bool:
        return module_id in self._rl_modules

    def __len__(self) -> int:
        return len(self._rl_modules)

    def __iter__(self):
        return iter(self._rl_modules.keys())

    # forward -----------------------------------------------------------------
    def _run(self, fn: str, batch: Dict[str, Dict]) -> Dict[str, Dict]:
        return {mid: getattr(self._rl_modules[mid], fn)(b) for mid, b in batch.items()}

    def forward_inference(self, batch):
        return self._run("forward_inference", batch)

    def forward_exploration(self, batch):
        return self._run("forward_exploration", batch)

    def forward_train(self, batch):
        return self._run("forward_train", batch)

    # state -------------------------------------------------------------------
    def get_state(self, module_ids: Optional[Iterable[str]] = None) -> Dict[str, Any]:
        ids = list(module_ids) if module_ids is not None else self.keys()
        return {mid: self._rl_modules[mid].get_state() for mid in ids}

    def set_state(self, state: Dict[str, Any]):
        for mid, st in state.items():
            if mid in self._rl_modules:
                self._rl_modules[mid].set_state(st)


@dataclass
class MultiRLModuleSpec:
    rl_module_specs: Dict[str, RLModuleSpec] = field(default_factory=dict)
    multi_rl_module_class: type = MultiRLModule

    def build(self, spaces: Dict[str, tuple], default_class=None, default_model_config=None) -> MultiRLModule:
        """``spaces``: module id -> (observation_space, action_space)."""
        mods = {}
        for mid, (obs, act) in spaces.items():
            spec = self.rl_module_specs.get(mid) or RLModuleSpec(default_class, dict(default_model_config or {}))
            if spec.module_class is None:
                spec = RLModuleSpec(default_class, {**dict(default_model_config or {}), **spec.model_config},
                                    spec.observation_space, spec.action_space)
            mods[mid] = spec.build(spec.observation_space or obs, spec.action_space or act)
        return self.multi_rl_module_class(mods)

    def module_factory(self, mid: str, default_class=None, default_model_config=None) -> Callable:
        spec = self.rl_module_specs.get(mid) or RLModuleSpec(default_class, {})
        cls = spec.module_class or default_class
        mc = {**dict(default_model_config or {}), **dict(spec.model_config or {})}
        return lambda obs, act: cls(spec.observation_space or obs, spec.action_space or act, mc)
