"""DQN (reference: rllib/algorithms/dqn/dqn.py, dqn_learner.py,
torch/dqn_torch_learner.py): epsilon-greedy EnvRunners, (prioritized) replay,
double-Q targets from a target network, Huber TD loss, optional dueling head."""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..core.learner import Learner, _to_tensor
from ..core.rl_module import NatureCNN, RLModule, _act, mlp
from ..env import Discrete
from .algorithm import Algorithm, AlgorithmConfig, OffPolicyMixin


class DQNModule(RLModule):
    def setup(self):
        mc = self.model_config
        assert isinstance(self.action_space, Discrete), "DQN needs a discrete action space"
        obs = self.observation_space
        self.image = len(obs.shape) == 3
        hiddens = list(mc.get("fcnet_hiddens", [256, 256]))
        if self.image:
            self.encoder = NatureCNN(obs.shape[-1], hw=obs.shape[:2])
            feat = self.encoder.out_dim
        else:
            self.encoder = mlp([int(np.prod(obs.shape))] + hiddens, _act(mc.get("fcnet_activation", "relu")),
                               out_act=True)
            feat = hiddens[-1]
        n = self.action_space.n
        self.dueling = mc.get("dueling", True)
        self.adv = nn.Linear(feat, n)
        self.val = nn.Linear(feat, 1) if self.dueling else None

    def q(self, obs):
        o = obs if self.image else obs.reshape(obs.shape[0], -1).float()
        z = self.encoder(o)
        a = self.adv(z)
        if self.dueling:
            return self.val(z) + a - a.mean(-1, keepdim=True)
        return a

    def forward_train(self, batch):
        return {"qf_preds": self.q(batch["obs"])}

    @torch.no_grad()
    def forward_inference(self, batch):
        return {"actions": self.q(batch["obs"]).argmax(-1)}

    @torch.no_grad()
    def forward_exploration(self, batch):
        q = self.q(batch["obs"])
        a = q.argmax(-1)
        eps = float(batch.get("epsilon", 0.0))
        if eps > 0:
            rnd = torch.randint(0, q.shape[-1], a.shape)
            mask = torch.rand(a.shape) < eps
            a = torch.where(mask, rnd, a)
        return {"actions": a}


class DQNConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class or DQN)
        self.lr = 5e-4
        self.train_batch_size = 32
        self.rollout_fragment_length = 4
        self.replay_buffer_config = {"type": "PrioritizedEpisodeReplayBuffer", "capacity": 50_000,
                                     "alpha": 0.6, "beta": 0.4}
        self.num_steps_sampled_before_learning_starts = 1000
        self.target_network_update_freq = 500
        self.double_q = True
        self.dueling = True
        self.n_step = 1
        self.epsilon = [(0, 1.0), (10_000, 0.05)]
        self.training_intensity = None
        self.td_error_loss_fn = "huber"
        self.grad_clip = 40.0
        self.tau = 1.0

    def default_module_class(self):
        return DQNModule

    def algo_model_config(self):
        mc = dict(self.model_config)
        mc.setdefault("dueling", self.dueling)
        return mc

    def module_factory(self):
        mc = self.algo_model_config()
        cls = self.rl_module_class or DQNModule
        return lambda o, a: cls(o, a, mc)

    def runner_config(self):
        d = super().runner_config()
        d["need_next_obs"] = True
        return d


class DQNLearner(Learner):
    def build(self):
        import copy

        self.target = copy.deepcopy(self.module)
        for p in self.target.parameters():
            p.requires_grad_(False)

    def compute_loss(self, batch):
        c = self.config
        q = self.module.forward_train(batch)["qf_preds"]
        q_sel = q.gather(-1, batch["actions"].long().unsqueeze(-1)).squeeze(-1)
        with torch.no_grad():
            q_next_t = self.target.q(batch["next_obs"])
            if c.get("double_q", True):
                a_star = self.module.q(batch["next_obs"]).argmax(-1, keepdim=True)
                q_next = q_next_t.gather(-1, a_star).squeeze(-1)
            else:
                q_next = q_next_t.max(-1).values
            target = batch["rewards"] + (c["gamma"] ** c.get("n_step", 1)) * (1 - batch["terminateds"]) * q_next
        td = q_sel - target
        if c.get("td_error_loss_fn", "huber") == "huber":
            l = F.smooth_l1_loss(q_sel, target, reduction="none")
        else:
            l = 0.5 * td ** 2
        loss = (batch["weights"] * l).mean()
        self._td = td.detach()
        return {"default": loss}, {"total_loss": loss.detach(), "qf_mean": q_sel.mean().detach(),
                                   "td_error_mean": td.abs().mean().detach()}

    def update_target(self):
        tau = self.config.get("tau", 1.0)
        with torch.no_grad():
            for pt, p in zip(self.target.parameters(), self.module.parameters()):
                pt.mul_(1 - tau).add_(p, alpha=tau)
        return True

    def train_on(self, batch):
        stats = self.update(batch)
        return stats, self._td.abs().cpu().numpy()

    def get_state(self):
        st = super().get_state()
        st["target"] = self.target.get_state()
        return st

    def set_state(self, st):
        super().set_state(st)
        if "target" in st:
            self.target.set_state(st["target"])
        return True


def _schedule(points, t):
    xs = [p[0] for p in points]
    ys = [p[1] for p in points]
    return float(np.interp(t, xs, ys))


class DQN(OffPolicyMixin, Algorithm):
    config_class = DQNConfig
    learner_class = DQNLearner
    supports_multi_agent = True

    def setup_algo(self):
        self.setup_replay()
        self._last_target = 0

    def _sync_weights(self, extra=None):
        c = self.algo_config
        eps = _schedule(c.epsilon, getattr(self, "env_steps_sampled", 0))
        super()._sync_weights({"epsilon": eps})

    def training_step(self):
        c = self.algo_config
        steps = self.sample_into_replay()
        stats = {}
        if self.replay_ready():
            # replay ratio: `training_intensity` trained / sampled steps (default 1 update per fragment)
            n_updates = 1 if not c.training_intensity else max(1, int(round(
                c.training_intensity * steps / c.train_batch_size)))
            for _ in range(n_updates):
                stats = self.replay_update()
            # target sync every `target_network_update_freq` sampled env steps
            if self.env_steps_sampled - self._last_target >= c.target_network_update_freq:
                self.learner_group.call("update_target")
                self._last_target = self.env_steps_sampled
        self._sync_weights()
        eps = _schedule(c.epsilon, self.env_steps_sampled)
        if self.is_multi_agent:
            for m in stats:
                stats[m]["epsilon"] = eps
        else:
            stats["epsilon"] = eps
        return stats
