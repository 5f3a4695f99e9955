"""``SampleBatch`` / ``MultiAgentBatch``: the old API stack's column batches
(reference role: rllib/policy/sample_batch.py:101, :1350).

A SampleBatch is a dict of equally long columns (numpy arrays, lists or torch
tensors). The new stack here trains from fragment dicts with the same column
names (``obs``, ``actions``, ``rewards``, ``terminateds`` ...), so a SampleBatch
IS a valid offline input (``config.offline_data(input_=[batch, ...])``), and
JSON lines written by :meth:`SampleBatch.to_json_lines` read back with
:meth:`SampleBatch.from_json_lines`."""
from __future__ import annotations

import json
from typing import Any, Dict, Iterator, List, Optional

import numpy as np

DEFAULT_POLICY_ID = "default_policy"


def _len(v) -> int:
    return int(v.shape[0]) if hasattr(v, "shape") and len(getattr(v, "shape", ())) else len(v)


def _take(v, idx):
    if isinstance(v, list):
        if isinstance(idx, slice):
            return v[idx]
        return [v[i] for i in idx]
    return v[idx]


def _cat(vals):
    first = vals[0]
    if isinstance(first, list):
        return [x for v in vals for x in v]
    try:
        import torch

        if isinstance(first, torch.Tensor):
            return torch.cat(vals)
    except ImportError:  # pragma: no cover
        pass
    return np.concatenate([np.asarray(v) for v in vals])


class SampleBatch(dict):
    OBS = "obs"
    NEXT_OBS = "new_obs"
    ACTIONS = "actions"
    REWARDS = "rewards"
    PREV_ACTIONS = "prev_actions"
    PREV_REWARDS = "prev_rewards"
    TERMINATEDS = "terminateds"
    TRUNCATEDS = "truncateds"
    INFOS = "infos"
    SEQ_LENS = "seq_lens"
    T = "t"
    EPS_ID = "eps_id"
    ENV_ID = "env_id"
    AGENT_INDEX = "agent_index"
    UNROLL_ID = "unroll_id"
    ACTION_DIST_INPUTS = "action_dist_inputs"
    ACTION_PROB = "action_prob"
    ACTION_LOGP = "action_logp"
    VF_PREDS = "vf_preds"
    VALUES_BOOTSTRAPPED = "values_bootstrapped"
    ADVANTAGES = "advantages"
    VALUE_TARGETS = "value_targets"

    def __init__(self, *args, **kwargs):
        self._is_training = bool(kwargs.pop("_is_training", False))
        super().__init__(*args, **kwargs)
        seq_lens = self.get(self.SEQ_LENS)
        cols = {k: _len(v) for k, v in self.items() if k != self.SEQ_LENS and _is_column(v)}
        lens = set(cols.values())
        if len(lens) > 1:
            raise ValueError(f"SampleBatch columns differ in length: {cols}")
        self.count = lens.pop() if lens else 0
        self._seq_lens = None if seq_lens is None else np.asarray(seq_lens)

    # ------------------------------------------------------------------ sizes
    def __len__(self) -> int:
        return self.count

    def agent_steps(self) -> int:
        return self.count

    def env_steps(self) -> int:
        return self.count

    def size_bytes(self) -> int:
        return int(sum(getattr(v, "nbytes", 0) for v in self.values()))

    # ------------------------------------------------------------ combination
    @staticmethod
    def concat_samples(samples: List["SampleBatch"]) -> "SampleBatch":
        samples = [s for s in samples if len(s)]
        if not samples:
            return SampleBatch()
        if any(isinstance(s, MultiAgentBatch) for s in samples):
            return MultiAgentBatch.concat_samples(samples)
        keys = [k for k in samples[0] if k != SampleBatch.SEQ_LENS]
        out = {k: _cat([s[k] for s in samples]) for k in keys}
        if all(s._seq_lens is not None for s in samples):
            out[SampleBatch.SEQ_LENS] = np.concatenate([s._seq_lens for s in samples])
        return SampleBatch(out)

    def concat(self, other: "SampleBatch") -> "SampleBatch":
        return SampleBatch.concat_samples([self, other])

    def copy(self, shallow: bool = False) -> "SampleBatch":
        return SampleBatch({k: (v if shallow else (v.copy() if hasattr(v, "copy") else list(v)))
                            for k, v in self.items()})

    # --------------------------------------------------------------- access
    def rows(self) -> Iterator[Dict[str, Any]]:
        for i in range(self.count):
            yield {k: v[i] for k, v in self.items() if k != self.SEQ_LENS}

    def columns(self, keys: List[str]) -> List[Any]:
        return [self[k] for k in keys]

    def slice(self, start: int, end: int) -> "SampleBatch":
        return SampleBatch({k: _take(v, slice(start, end)) for k, v in self.items() if k != self.SEQ_LENS})

    def __getitem__(self, key):
        if isinstance(key, slice):
            return self.slice(key.start or 0, self.count if key.stop is None else key.stop)
        return dict.__getitem__(self, key)

    def shuffle(self, seed: Optional[int] = None) -> "SampleBatch":
        perm = np.random.default_rng(seed).permutation(self.count)
        for k in list(self):
            if k != self.SEQ_LENS:
                dict.__setitem__(self, k, _take(self[k], perm))
        return self

    def split_by_episode(self, key: Optional[str] = None) -> List["SampleBatch"]:
        """One batch per episode: by ``eps_id`` when present, else cut after every
        terminated / truncated step."""
        key = key or (self.EPS_ID if self.EPS_ID in self else None)
        if key is not None:
            ids = np.asarray(self[key])
            cuts = [0] + [i for i in range(1, self.count) if ids[i] != ids[i - 1]] + [self.count]
        else:
            done = np.zeros(self.count, bool)
            for k in (self.TERMINATEDS, self.TRUNCATEDS, "dones"):
                if k in self:
                    done |= np.asarray(self[k]).astype(bool)
            cuts = [0] + [i + 1 for i in np.nonzero(done)[0] if i + 1 < self.count] + [self.count]
        return [self.slice(a, b) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]

    def timeslices(self, size: Optional[int] = None, num_slices: Optional[int] = None,
                   k: Optional[int] = None) -> List["SampleBatch"]:
        size = size or k or -(-self.count // max(1, num_slices or 1))
        return [self.slice(s, min(self.count, s + size)) for s in range(0, self.count, size)]

    def to_device(self, device, framework: str = "torch") -> "SampleBatch":
        import torch

        for k, v in list(self.items()):
            if isinstance(v, np.ndarray) and v.dtype != object:
                dict.__setitem__(self, k, torch.as_tensor(v, device=device))
            elif isinstance(v, torch.Tensor):
                dict.__setitem__(self, k, v.to(device))
        return self

    def as_multi_agent(self, module_id: Optional[str] = None) -> "MultiAgentBatch":
        return MultiAgentBatch({module_id or DEFAULT_POLICY_ID: self}, self.count)

    def is_training(self) -> bool:
        return self._is_training

    def set_training(self, training: bool = True):
        self._is_training = bool(training)

    def get_single_step_input_dict(self, view_requirements=None, index: int = -1) -> "SampleBatch":
        i = index if index >= 0 else self.count + index
        return SampleBatch({k: _take(v, slice(i, i + 1)) for k, v in self.items() if k != self.SEQ_LENS})

    # ---------------------------------------------------------------- fragments
    def to_fragment(self) -> Dict[str, np.ndarray]:
        """The new stack's fragment columns (numpy)."""
        out = {k: np.asarray(v) for k, v in self.items() if k not in (self.SEQ_LENS, self.INFOS)}
        if self.NEXT_OBS in out and "next_obs" not in out:
            out["next_obs"] = out.pop(self.NEXT_OBS)
        return out

    # ---------------------------------------------------------------- JSON
    def to_json_lines(self) -> str:
        """One JSON object per row (the offline JSON writer's row format)."""
        def plain(x):
            return x.tolist() if isinstance(x, np.ndarray) else (x.item() if isinstance(x, np.generic) else x)

        return "\n".join(json.dumps({k: plain(v) for k, v in r.items()}) for r in self.rows())

    @staticmethod
    def from_json_lines(text: str) -> "SampleBatch":
        rows = [json.loads(ln) for ln in text.splitlines() if ln.strip()]
        if not rows:
            return SampleBatch()
        if rows[0].get("type") == "SampleBatch":  # the reference's whole-batch-per-line form
            return SampleBatch.concat_samples([SampleBatch({k: np.asarray(v) for k, v in r.items() if k != "type"})
                                               for r in rows])
        return SampleBatch({k: np.asarray([r[k] for r in rows]) for k in rows[0]})

    def __repr__(self):
        return f"SampleBatch({self.count}: {list(self.keys())})"


def _is_column(v) -> bool:
    return isinstance(v, (list, np.ndarray)) or hasattr(v, "shape")


class MultiAgentBatch:
    """Per-module SampleBatches of one stretch of multi-agent experience."""

    def __init__(self, policy_batches: Dict[str, SampleBatch], env_steps: int):
        self.policy_batches = dict(policy_batches)
        self.count = int(env_steps)

    def env_steps(self) -> int:
        return self.count

    def agent_steps(self) -> int:
        return sum(len(b) for b in self.policy_batches.values())

    def __len__(self) -> int:
        return self.count

    def __getitem__(self, key: str) -> SampleBatch:
        return self.policy_batches[key]

    @staticmethod
    def wrap_as_needed(policy_batches: Dict[str, SampleBatch], env_steps: int):
        if len(policy_batches) == 1 and DEFAULT_POLICY_ID in policy_batches:
            return policy_batches[DEFAULT_POLICY_ID]
        return MultiAgentBatch(policy_batches, env_steps)

    @staticmethod
    def concat_samples(samples: List[Any]) -> "MultiAgentBatch":
        parts: Dict[str, List[SampleBatch]] = {}
        steps = 0
        for s in samples:
            s = s.as_multi_agent() if isinstance(s, SampleBatch) else s
            for pid, b in s.policy_batches.items():
                parts.setdefault(pid, []).append(b)
            steps += s.count
        return MultiAgentBatch({p: SampleBatch.concat_samples(bs) for p, bs in parts.items()}, steps)

    def copy(self) -> "MultiAgentBatch":
        return MultiAgentBatch({p: b.copy() for p, b in self.policy_batches.items()}, self.count)

    def size_bytes(self) -> int:
        return sum(b.size_bytes() for b in self.policy_batches.values())

    def as_multi_agent(self) -> "MultiAgentBatch":
        return self

    def to_device(self, device, framework: str = "torch") -> "MultiAgentBatch":
        for b in self.policy_batches.values():
            b.to_device(device, framework)
        return self

    def __repr__(self):
        return f"MultiAgentBatch({self.count}: {list(self.policy_batches)})"


def concat_samples(samples):
    return SampleBatch.concat_samples(samples)
