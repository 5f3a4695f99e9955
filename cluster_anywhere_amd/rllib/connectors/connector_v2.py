"""ConnectorV2 and connector pipelines (reference role: rllib/connectors/connector_v2.py:31,
connector_pipeline_v2.py).

A connector is a callable piece that transforms a ``batch`` dict on one of the
three data paths:

* env -> module (on env runners): raw env observations -> module inputs
  (``batch["obs"]``: numpy ``[B, ...]``; ``episodes``: the B episode records);
* module -> env (on env runners): module outputs -> env actions
  (``batch["actions_for_env"]``);
* learner (on learners): a time-major sample fragment -> the train batch
  (GAE, flattening, masking).

Every call is ``connector(rl_module=..., batch=..., episodes=..., explore=...,
shared_data=..., metrics=...)`` and returns the (new) batch. Connectors that
change the observation shape report it through
``recompute_output_observation_space`` so the RLModule is built for what it
will actually receive. ``get_state``/``set_state`` carry learned statistics
(e.g. running mean/std), and ``merge_states`` combines the states of the same
connector on several env runners.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence, Type, Union


class ConnectorV2:
    def __init__(self, input_observation_space=None, input_action_space=None, **kwargs):
        self.input_observation_space = input_observation_space
        self.input_action_space = input_action_space

    # spaces ------------------------------------------------------------------
    def recompute_output_observation_space(self, input_observation_space, input_action_space):
        return input_observation_space

    def recompute_output_action_space(self, input_observation_space, input_action_space):
        return input_action_space

    @property
    def observation_space(self):
        return self.recompute_output_observation_space(self.input_observation_space, self.input_action_space)

    @property
    def action_space(self):
        return self.recompute_output_action_space(self.input_observation_space, self.input_action_space)

    # call --------------------------------------------------------------------
    def __call__(self, *, rl_module=None, batch: Dict[str, Any], episodes: Sequence = (), explore: Optional[bool] = None,
                 shared_data: Optional[Dict] = None, metrics=None, **kwargs) -> Dict[str, Any]:
        raise NotImplementedError

    # state -------------------------------------------------------------------
    def get_state(self) -> Dict[str, Any]:
        return {}

    def set_state(self, state: Dict[str, Any]) -> None:
        pass

    def reset_state(self) -> None:
        pass

    def episode_done(self, episode) -> None:
        """Called by the env runner when ``episode`` has finished (drop per-episode state)."""

    @staticmethod
    def merge_states(states: List[Dict[str, Any]]) -> Dict[str, Any]:
        return states[0] if states else {}

    @property
    def name(self) -> str:
        return type(self).__name__

    def __repr__(self):
        return f"{self.name}()"


class ConnectorPipelineV2(ConnectorV2):
    """An ordered list of connectors run one after another (itself a connector)."""

    def __init__(self, input_observation_space=None, input_action_space=None,
                 connectors: Optional[Sequence[ConnectorV2]] = None, **kwargs):
        super().__init__(input_observation_space, input_action_space)
        self.connectors: List[ConnectorV2] = []
        for c in connectors or ():
            self.append(c)

    # structure ---------------------------------------------------------------
    def _fix_spaces(self):
        obs, act = self.input_observation_space, self.input_action_space
        for c in self.connectors:
            c.input_observation_space, c.input_action_space = obs, act
            obs = c.recompute_output_observation_space(obs, act)
            act = c.recompute_output_action_space(obs, act)

    def set_input_spaces(self, obs_space, act_space):
        self.input_observation_space, self.input_action_space = obs_space, act_space
        self._fix_spaces()

    def _index(self, name_or_class: Union[str, Type]) -> int:
        for i, c in enumerate(self.connectors):
            if (isinstance(name_or_class, str) and c.name == name_or_class) or \
                    (isinstance(name_or_class, type) and isinstance(c, name_or_class)):
                return i
        raise ValueError(f"no connector {name_or_class!r} in {self}")

    def append(self, connector: ConnectorV2) -> "ConnectorPipelineV2":
        self.connectors.append(connector)
        self._fix_spaces()
        return self

    def prepend(self, connector: ConnectorV2) -> "ConnectorPipelineV2":
        self.connectors.insert(0, connector)
        self._fix_spaces()
        return self

    def insert_before(self, name_or_class, connector: ConnectorV2) -> ConnectorV2:
        self.connectors.insert(self._index(name_or_class), connector)
        self._fix_spaces()
        return connector

    def insert_after(self, name_or_class, connector: ConnectorV2) -> ConnectorV2:
        self.connectors.insert(self._index(name_or_class) + 1, connector)
        self._fix_spaces()
        return connector

    def remove(self, name_or_class) -> None:
        del self.connectors[self._index(name_or_class)]
        self._fix_spaces()

    def __len__(self) -> int:
        return len(self.connectors)

    def __iter__(self):
        return iter(self.connectors)

    def __getitem__(self, i):
        if isinstance(i, (str, type)):
            return self.connectors[self._index(i)]
        return self.connectors[i]

    def recompute_output_observation_space(self, input_observation_space, input_action_space):
        obs, act = input_observation_space, input_action_space
        for c in self.connectors:
            obs, act = c.recompute_output_observation_space(obs, act), c.recompute_output_action_space(obs, act)
        return obs

    def recompute_output_action_space(self, input_observation_space, input_action_space):
        obs, act = input_observation_space, input_action_space
        for c in self.connectors:
            obs, act = c.recompute_output_observation_space(obs, act), c.recompute_output_action_space(obs, act)
        return act

    # call --------------------------------------------------------------------
    def __call__(self, *, rl_module=None, batch, episodes=(), explore=None, shared_data=None, metrics=None,
                 **kwargs):
        shared_data = {} if shared_data is None else shared_data
        for c in self.connectors:
            out = c(rl_module=rl_module, batch=batch, episodes=episodes, explore=explore, shared_data=shared_data,
                    metrics=metrics, **kwargs)
            if out is not None:
                batch = out
        return batch

    # state -------------------------------------------------------------------
    def get_state(self):
        return {f"{i}:{c.name}": c.get_state() for i, c in enumerate(self.connectors)}

    def set_state(self, state):
        for i, c in enumerate(self.connectors):
            k = f"{i}:{c.name}"
            if k in state:
                c.set_state(state[k])

    def reset_state(self):
        for c in self.connectors:
            c.reset_state()

    def episode_done(self, episode):
        for c in self.connectors:
            c.episode_done(episode)

    def merge_states(self, states: List[Dict[str, Any]]) -> Dict[str, Any]:  # type: ignore[override]
        out = {}
        for i, c in enumerate(self.connectors):
            k = f"{i}:{c.name}"
            sub = [s[k] for s in states if k in s]
            if sub:
                out[k] = c.merge_states(sub)
        return out

    def __repr__(self):
        return f"ConnectorPipelineV2({', '.join(c.name for c in self.connectors)})"


def build_pipeline(spec, env=None, obs_space=None, act_space=None) -> ConnectorPipelineV2:
    """Pipeline from a user spec: a connector, a list of connectors, or a
    callable ``(env)`` / ``(obs_space, act_space)`` returning either."""
    items = spec
    if callable(spec) and not isinstance(spec, ConnectorV2):
        try:
            items = spec(env) if obs_space is None else spec(obs_space, act_space)
        except TypeError:
            items = spec(obs_space, act_space) if obs_space is None else spec(env)
    if items is None:
        items = []
    if isinstance(items, ConnectorPipelineV2):
        p = items
    else:
        p = ConnectorPipelineV2(connectors=list(items) if isinstance(items, (list, tuple)) else [items])
    return p
