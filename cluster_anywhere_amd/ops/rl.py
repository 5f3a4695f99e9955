"""GAE and V-trace return estimators (``rl_returns.hip``), time-major [T, B]."""
from __future__ import annotations

import torch

from ._lib import kernels, use_gpu_kernel


def gae_ref(rewards, values, nonterminal, gamma, lam):
    T = rewards.shape[0]
    adv = torch.zeros_like(rewards)
    a = torch.zeros_like(rewards[0])
    for t in range(T - 1, -1, -1):
        delta = rewards[t] + gamma * values[t + 1] * nonterminal[t] - values[t]
        a = delta + gamma * lam * nonterminal[t] * a
        adv[t] = a
    return adv, adv + values[:T]


def gae(rewards, values, nonterminal, gamma=0.99, lam=0.95):
    """rewards/nonterminal: [T, B]; values: [T+1, B] (last row = bootstrap)."""
    if use_gpu_kernel(rewards, values, nonterminal):
        return tuple(
            kernels().gae(
                rewards.float().contiguous(),
                values.float().contiguous(),
                nonterminal.float().contiguous(),
                gamma,
                lam,
            )
        )
    return gae_ref(rewards.float(), values.float(), nonterminal.float(), gamma, lam)


def vtrace_ref(log_rhos, discounts, rewards, values, bootstrap, clip_rho=1.0, clip_pg_rho=1.0):
    rhos = torch.exp(log_rhos)
    crho = torch.clamp(rhos, max=clip_rho) if clip_rho and clip_rho > 0 else rhos
    cs = torch.clamp(rhos, max=1.0)
    v_tp1 = torch.cat([values[1:], bootstrap[None]], 0)
    deltas = crho * (rewards + discounts * v_tp1 - values)
    acc = torch.zeros_like(bootstrap)
    out = []
    for t in range(values.shape[0] - 1, -1, -1):
        acc = deltas[t] + discounts[t] * cs[t] * acc
        out.append(acc)
    vs_minus_v = torch.stack(out[::-1], 0)
    vs = vs_minus_v + values
    vs_tp1 = torch.cat([vs[1:], bootstrap[None]], 0)
    cpg = torch.clamp(rhos, max=clip_pg_rho) if clip_pg_rho and clip_pg_rho > 0 else rhos
    pg = cpg * (rewards + discounts * vs_tp1 - values)
    return vs, pg


def vtrace(log_rhos, discounts, rewards, values, bootstrap, clip_rho=1.0, clip_pg_rho=1.0):
    if use_gpu_kernel(log_rhos, discounts, rewards, values, bootstrap):
        f = lambda t: t.float().contiguous()
        return tuple(
            kernels().vtrace(
                f(log_rhos), f(discounts), f(rewards), f(values), f(bootstrap), clip_rho, clip_pg_rho
            )
        )
    return vtrace_ref(log_rhos, discounts, rewards, values, bootstrap, clip_rho, clip_pg_rho)
