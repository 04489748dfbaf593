"""Evaluation: greedy rollouts of the population / frozen path of a checkpoint.

The reference has a display path (``run_policy``, ``game_ac_network.py:458-465``,
and ``GameState(display=True)`` with a gym Monitor).  Here evaluation runs the
whole population on device, one env per path, argmax actions, until each path
finished ``episodes`` episodes or ``max_steps`` steps.
"""
from __future__ import annotations

import numpy as np
import torch

from ..envs.registry import make
from ..models.acnet import ACPathNet


@torch.no_grad()
def evaluate_model(model: ACPathNet, env_id: str, episodes: int = 1, max_steps: int = 2000, device="cpu",
                   seed: int = 12345, frameskip: int = 4, gray: str = "rgb", sample: bool = False):
    """Mean return per path over ``episodes`` episodes (NaN for a path that finished none in ``max_steps``).
    ``sample=False`` plays the argmax action; ``sample=True`` samples the policy with a seeded generator,
    so a repeated evaluation of unchanged parameters replays the same episodes."""
    P = model.P
    gen = torch.Generator(device=device).manual_seed(seed) if sample else None
    kw = {} if env_id.startswith("CartPole") else dict(frameskip=frameskip, gray=gray)
    env = make(env_id, num_envs=P, device=device, seed=seed, backend="torch", **kw)
    obs = env.reset()
    state = model.init_state(P)
    returns = [[] for _ in range(P)]
    for _ in range(max_steps):
        logits, value, state = model.forward(obs, 1, state)
        if sample:
            a = torch.multinomial(torch.softmax(logits.float(), -1), 1, generator=gen).reshape(-1)
        else:
            a = logits.argmax(-1)
        obs, r, d, info = env.step(a)
        if state is not None:
            keep = (~d).float()[:, None]
            state = (state[0] * keep, state[1] * keep)
        for p in np.nonzero(d.cpu().numpy())[0]:
            returns[p].append(float(info["episode_return"][p]))
        if all(len(x) >= episodes for x in returns):
            break
    return [float(np.mean(x)) if x else float("nan") for x in returns]


def evaluate_checkpoint(cfg, path: str, episodes: int = 1, max_steps: int = 2000, device="cpu"):
    from safetensors.torch import load_file
    d = load_file(path)
    g = d["ga.genotypes"].numpy().astype(np.float32)
    fr = d["ga.frozen"].numpy().astype(np.float32)
    P = g.shape[0]
    model = ACPathNet(cfg.net, P, device, "torch")
    st = model.store
    with torch.no_grad():
        for s in st.layout.segments:
            st.flat[s.offset:s.offset + s.numel].copy_(d[s.name].reshape(-1))
    expr = ((g > 0.5) | (fr[None] > 0.5)).astype(np.float32)
    model.set_paths(expr)
    task = int(d["train.task_idx"][0])
    model.task = task
    env_id = cfg.tasks[min(task, len(cfg.tasks) - 1)]
    rets = evaluate_model(model, env_id, episodes, max_steps, device, frameskip=cfg.frameskip, gray=cfg.gray)
    return {"env": env_id, "task": task, "returns": rets, "best_path": int(np.nanargmax(rets)) if rets else -1,
            "best_return": float(np.nanmax(rets)) if rets else float("nan")}
