"""Episode recording for offline RL: ``config.offline_data(output=path)``.

Role of the reference's ``OfflineSingleAgentEnvRunner``
(``rllib/offline/offline_env_runner.py:30,122``): every env runner of an on-policy
algorithm writes what it samples to Parquet under ``output``, one row per env step,
so a later BC / MARWIL / CQL run (or an off-policy estimate) can read it back.

Design: rows are buffered PER EPISODE inside the runner and committed to the file
buffer only when the episode ends (``output_write_episodes=True``, the default), so
every file holds whole episodes. The offline reader then maps each file as one block
and can compute per-episode quantities (discounted returns, importance ratios)
without ever seeing half an episode. Unfinished episodes at ``stop()`` are written
as truncated. Columns (:data:`COLUMNS`): ``eps_id`` (``<runner>-<env>-<n>``), ``t``,
``obs``, ``new_obs``, ``actions``, ``rewards``, ``terminateds``, ``truncateds``,
``action_logp`` and ``action_prob`` of the behaviour policy (for importance
sampling), ``vf_preds`` when the module has a value head.
"""
from __future__ import annotations

import os
import threading
from typing import Dict, List, Optional

import numpy as np

COLUMNS = ("eps_id", "t", "obs", "new_obs", "actions", "rewards", "terminateds", "truncateds",
           "action_logp", "action_prob", "vf_preds")


class EpisodeRecorder:
    """Buffers env-runner steps per (env, episode) and writes whole episodes to
    ``<output>/run-<runner>-<file>.parquet`` once ``max_rows_per_file`` rows are
    pending (and on :meth:`flush`)."""

    def __init__(self, output: str, worker_index: int, num_envs: int, max_rows_per_file: int = 10_000,
                 write_episodes: bool = True):
        self.output = output
        self.worker_index = int(worker_index)
        self.max_rows = max(1, int(max_rows_per_file))
        self.write_episodes = write_episodes
        os.makedirs(output, exist_ok=True)
        self._open: List[Dict[str, list]] = [self._empty() for _ in range(num_envs)]
        self._eps_n = [0] * num_envs
        self._ids = [self._eps_id(i) for i in range(num_envs)]
        self._t = [0] * num_envs
        self._ready: Dict[str, list] = self._empty()
        self._rows = 0
        self._files = 0
        self._lock = threading.Lock()
        self.files_written: List[str] = []

    @staticmethod
    def _empty() -> Dict[str, list]:
        return {k: [] for k in COLUMNS}

    def _eps_id(self, env: int) -> str:
        return f"{self.worker_index}-{env}-{self._eps_n[env]}"

    def add_step(self, env: int, obs, new_obs, action, reward, terminated: bool, truncated: bool,
                 logp: Optional[float], vf: Optional[float]):
        buf = self._open[env]
        buf["eps_id"].append(self._ids[env])
        buf["t"].append(self._t[env])
        buf["obs"].append(np.asarray(obs, dtype=np.float32))
        buf["new_obs"].append(np.asarray(new_obs, dtype=np.float32))
        buf["actions"].append(np.asarray(action))
        buf["rewards"].append(float(reward))
        buf["terminateds"].append(bool(terminated))
        buf["truncateds"].append(bool(truncated))
        lp = float("nan") if logp is None else float(logp)
        buf["action_logp"].append(lp)
        buf["action_prob"].append(float(np.exp(lp)) if logp is not None else float("nan"))
        buf["vf_preds"].append(float("nan") if vf is None else float(vf))
        self._t[env] += 1
        if terminated or truncated:
            self._commit(env)
        elif not self.write_episodes:
            self._commit(env, close=False)

    def _commit(self, env: int, close: bool = True):
        buf = self._open[env]
        n = len(buf["t"])
        if n:
            with self._lock:
                for k in COLUMNS:
                    self._ready[k].extend(buf[k])
                self._rows += n
            self._open[env] = self._empty()
        if close:
            self._eps_n[env] += 1
            self._ids[env] = self._eps_id(env)
            self._t[env] = 0
        if self._rows >= self.max_rows:
            self.flush()

    def flush(self, include_open: bool = False) -> Optional[str]:
        """Write the committed rows (and, with ``include_open``, every unfinished
        episode, marked truncated at its last step) to a new Parquet file."""
        if include_open:
            for env, buf in enumerate(self._open):
                if buf["t"]:
                    buf["truncateds"][-1] = True
                    self._commit(env)
        with self._lock:
            if not self._rows:
                return None
            cols, self._ready, self._rows = self._ready, self._empty(), 0
            path = os.path.join(self.output, f"run-{self.worker_index:03d}-{self._files:05d}.parquet")
            self._files += 1
        import pyarrow.parquet as pq

        from ...data.block import to_arrow

        block = {"eps_id": np.asarray(cols["eps_id"], dtype=object), "t": np.asarray(cols["t"], dtype=np.int64),
                 "obs": np.stack(cols["obs"]), "new_obs": np.stack(cols["new_obs"]),
                 "actions": np.stack(cols["actions"]),
                 "rewards": np.asarray(cols["rewards"], dtype=np.float32),
                 "terminateds": np.asarray(cols["terminateds"], dtype=bool),
                 "truncateds": np.asarray(cols["truncateds"], dtype=bool),
                 "action_logp": np.asarray(cols["action_logp"], dtype=np.float32),
                 "action_prob": np.asarray(cols["action_prob"], dtype=np.float32),
                 "vf_preds": np.asarray(cols["vf_preds"], dtype=np.float32)}
        tmp = path + ".tmp"
        pq.write_table(to_arrow(block), tmp)
        os.replace(tmp, path)  # readers never see a half-written file
        self.files_written.append(path)
        return path
