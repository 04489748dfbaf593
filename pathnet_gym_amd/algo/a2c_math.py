"""A2C math: n-step / GAE returns and the reference actor-critic loss.

Reference: ``a3c_training_thread.py:155-180`` (n-step return, reward clip),
``game_ac_network.py:20-59`` (loss).  These torch versions are the oracle
for the fused HIP kernels ``returns_scan`` and ``a2c_head_loss``.
"""
from __future__ import annotations

import torch


def nstep_returns(rewards: torch.Tensor, values: torch.Tensor, dones: torch.Tensor,
                  bootstrap: torch.Tensor, gamma: float, lam: float = 1.0, reward_clip: float = 1.0):
    """Reverse scan over T.

    rewards, values, dones: [T, B]; bootstrap: [B] = V(s_T).
    ``dones[t]`` means the episode ended AT step t (so s_{t+1} is a fresh
    episode and nothing bootstraps across it).  With lam=1 this is exactly the
    reference: R <- clip(r,-1,1) + gamma*R, td = R - V (R=0 at a terminal).
    Returns (R [T,B], adv [T,B]).
    """
    T = rewards.shape[0]
    r = rewards.clamp(-reward_clip, reward_clip) if reward_clip > 0 else rewards
    R = bootstrap
    gae = torch.zeros_like(bootstrap)
    next_v = bootstrap
    Rs, As = [], []
    for t in range(T - 1, -1, -1):
        nd = 1.0 - dones[t].float()
        if lam == 1.0:
            R = r[t] + gamma * R * nd
            Rs.append(R)
            As.append(R - values[t])
        else:
            delta = r[t] + gamma * next_v * nd - values[t]
            gae = delta + gamma * lam * nd * gae
            As.append(gae)
            Rs.append(gae + values[t])
            next_v = values[t]
    Rs.reverse()
    As.reverse()
    return torch.stack(Rs), torch.stack(As)


def a2c_loss(logits: torch.Tensor, values: torch.Tensor, actions: torch.Tensor,
             returns: torch.Tensor, adv: torch.Tensor, entropy_beta: float, value_coef: float = 0.5,
             weight: torch.Tensor | None = None):
    """Reference loss (sum over samples).

    logits [N, A], values [N], actions [N] long, returns/adv [N] (stop-grad).
    log_pi = log(clip(softmax, 1e-20, 1))       (game_ac_network.py:38)
    entropy = -sum pi*log_pi                       (:41)
    policy_loss = -sum(log_pi[a]*td + beta*entropy)   (:49)
    value_loss = value_coef * l2_loss(R - V) = value_coef*0.5*sum (R-V)^2   (:56)
    ``weight`` [N] optionally scales each sample (mean-over-envs reduction).
    """
    wide = logits.dtype == torch.float64            # float64 oracles (tests/test_x3_engine.py) stay float64
    pi = torch.softmax(logits if wide else logits.float(), -1)
    log_pi = torch.log(pi.clamp(1e-20, 1.0))
    entropy = -(pi * log_pi).sum(-1)
    lp_a = log_pi.gather(1, actions.long()[:, None]).squeeze(1)
    pol = -(lp_a * adv.detach() + entropy_beta * entropy)
    val = value_coef * 0.5 * (returns.detach() - (values if wide else values.float())) ** 2
    if weight is not None:
        pol = pol * weight
        val = val * weight
    return pol.sum() + val.sum(), pol.sum().detach(), val.sum().detach(), entropy.mean().detach()


def sample_actions(logits: torch.Tensor, generator=None) -> torch.Tensor:
    """Categorical sampling (a3c_training_thread.py:89-90), on device."""
    probs = torch.softmax(logits.float(), -1)
    return torch.multinomial(probs, 1, generator=generator).squeeze(1)


def sampling_u01(seed: int, stepkey: int, rows: torch.Tensor, A: int) -> torch.Tensor:
    """The uniforms of the HIP heads kernel's Gumbel-max (csrc/heads.hip u01), bit for bit: hash(stepkey * 64 +
    action) -> ^ global row -> ^ seed, 24 bits, centred.  rows: int64 [N] global sample indices.  [N, A] fp32."""
    from ..envs.base import wang_hash
    m = 0xFFFFFFFF
    j = torch.arange(A, dtype=torch.int64, device=rows.device)
    h = wang_hash(torch.full_like(j, (stepkey * 64) & m) + j)[None, :]        # [1, A]
    h = wang_hash(h ^ (rows[:, None] & m))
    h = wang_hash(h ^ (seed & m))
    return ((h >> 8).to(torch.float32) + 0.5) * (1.0 / 16777216.0)


def sample_actions_keyed(logits: torch.Tensor, seed: int, stepkey: int, row_base: int = 0,
                         greedy: bool = False) -> torch.Tensor:
    """Categorical sampling by Gumbel-max on the counter-based key (seed, stepkey, global row, action), the same
    draws as the HIP heads kernel.  Row b of ``logits`` is global sample row_base + b, so a population sharded
    over ranks samples exactly what one process sampling all rows would (strong scaling, TrainConfig.paths_total)."""
    lg = logits.detach().float()
    if greedy:
        return lg.argmax(-1)
    rows = torch.arange(lg.shape[0], dtype=torch.int64, device=lg.device) + int(row_base)
    u = sampling_u01(int(seed), int(stepkey), rows, lg.shape[1])
    return (lg - torch.log(-torch.log(u))).argmax(-1)
