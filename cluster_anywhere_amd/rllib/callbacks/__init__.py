"""RLlib callbacks (reference role: rllib/callbacks/callbacks.py:35 ``RLlibCallback``).

Hooks run in the component that owns the event: episode / sample hooks in the
env runner processes, algorithm hooks in the driver. Every hook receives
keyword arguments only, so subclasses can take just what they need (``**kw``).
Custom metrics go through ``metrics_logger.log_value(...)``; the env runner
group merges the runner loggers into ``result["env_runners"]``.

``config.callbacks(MyCallback)`` takes a class (or a list of classes); the
keyword form ``config.callbacks(on_episode_end=fn, ...)`` wraps plain
functions (the reference's ``on_*`` arguments of ``AlgorithmConfig.callbacks``).
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence, Type

HOOKS = ("on_algorithm_init", "on_train_result", "on_evaluate_start", "on_evaluate_end",
         "on_checkpoint_loaded", "on_env_runners_recreated", "on_environment_created",
         "on_episode_created", "on_episode_start", "on_episode_step", "on_episode_end", "on_sample_end")


class RLlibCallback:
    # --- algorithm (driver) -------------------------------------------------
    def on_algorithm_init(self, *, algorithm, metrics_logger=None, **kwargs):
        pass

    def on_train_result(self, *, algorithm, metrics_logger=None, result: Dict, **kwargs):
        pass

    def on_evaluate_start(self, *, algorithm, metrics_logger=None, **kwargs):
        pass

    def on_evaluate_end(self, *, algorithm, metrics_logger=None, evaluation_metrics: Dict, **kwargs):
        pass

    def on_checkpoint_loaded(self, *, algorithm, **kwargs):
        pass

    def on_env_runners_recreated(self, *, algorithm, env_runner_group, env_runner_indices: List[int], **kwargs):
        pass

    # --- env runner ---------------------------------------------------------
    def on_environment_created(self, *, env_runner, metrics_logger=None, env, env_context: Dict, **kwargs):
        pass

    def on_episode_created(self, *, episode, env_runner=None, metrics_logger=None, env=None, env_index: int = 0,
                           rl_module=None, **kwargs):
        pass

    def on_episode_start(self, *, episode, env_runner=None, metrics_logger=None, env=None, env_index: int = 0,
                         rl_module=None, **kwargs):
        pass

    def on_episode_step(self, *, episode, env_runner=None, metrics_logger=None, env=None, env_index: int = 0,
                        rl_module=None, **kwargs):
        pass

    def on_episode_end(self, *, episode, env_runner=None, metrics_logger=None, env=None, env_index: int = 0,
                       rl_module=None, **kwargs):
        pass

    def on_sample_end(self, *, env_runner=None, metrics_logger=None, samples=None, **kwargs):
        pass


DefaultCallbacks = RLlibCallback


class _Multi(RLlibCallback):
    """Fans every hook out to several callback objects (list form of ``config.callbacks``)."""

    def __init__(self, cbs: Sequence[RLlibCallback]):
        self._cbs = list(cbs)
        for h in HOOKS:
            setattr(self, h, self._fan(h))

    def _fan(self, hook):
        def call(**kw):
            for c in self._cbs:
                getattr(c, hook)(**kw)
        return call


class _Functions(RLlibCallback):
    def __init__(self, fns: Dict[str, Callable]):
        for h, fn in fns.items():
            if h not in HOOKS:
                raise ValueError(f"unknown callback hook {h!r}")
            setattr(self, h, (lambda f: (lambda **kw: f(**kw)))(fn))


def make_callbacks(callbacks_class=None, functions: Optional[Dict[str, Callable]] = None) -> RLlibCallback:
    """Instantiate what ``config.callbacks(...)`` recorded."""
    cbs: List[RLlibCallback] = []
    classes = callbacks_class if isinstance(callbacks_class, (list, tuple)) else [callbacks_class]
    for c in classes:
        if c is None:
            continue
        cbs.append(c() if isinstance(c, type) else c)
    if functions:
        cbs.append(_Functions(functions))
    if not cbs:
        return RLlibCallback()
    return cbs[0] if len(cbs) == 1 else _Multi(cbs)


__all__ = ["RLlibCallback", "DefaultCallbacks", "make_callbacks", "HOOKS"]
