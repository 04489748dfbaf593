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
    pi = torch.softmax(logits.float(), -1)
    log_pi = torch.log(pi.clamp(1e-20, 1.0))
    entropy = -(pi * log_pi).sum(-1)
    lp_a = log_pi.gather(1, actions.long()[:, None]).squeeze(1)
    pol = -(lp_a * adv.detach() + entropy_beta * entropy)
    val = value_coef * 0.5 * (returns.detach() - values.float()) ** 2
    if weight is not None:
        pol = pol * weight
        val = val * weight
    return pol.sum() + val.sum(), pol.sum().detach(), val.sum().detach(), entropy.mean().detach()


def sample_actions(logits: torch.Tensor, generator=None) -> torch.Tensor:
    """Categorical sampling (a3c_training_thread.py:89-90), on device."""
    probs = torch.softmax(logits.float(), -1)
    return torch.multinomial(probs, 1, generator=generator).squeeze(1)
