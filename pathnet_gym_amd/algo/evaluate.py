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


@torch.no_grad()
def evaluate_path(net_cfg, flat: torch.Tensor, expressed: np.ndarray, env_id: str, task: int = 0,
                  episodes: int = 64, seed: int = 424242, device="cpu", frameskip: int = 4, gray: str = "rgb",
                  max_steps: int = 30000, check_every: int = 32) -> dict:
    """Held-out evaluation of ONE path of a trained super-network: ``episodes`` fresh envs (their own seed, none of
    the training envs), each playing exactly one episode under the SAMPLED policy (seeded multinomial, so a repeat
    replays the same episodes) of the path ``expressed`` [L, M] with the weights ``flat`` (copied, never trained).
    The forward is the fp32 PyTorch oracle (models/pathnet.py trunk_forward_ref): independent of the HIP kernels
    that produced the training fitness (the env steps in its HIP kernel on a GPU).  The reference's equivalent is its display path (run_policy,
    game_ac_network.py:458-465); it has no held-out check of a tournament winner.

    Returns {"mean", "min", "max", "finished", "episodes", "steps", "returns"}; an env that finished no episode in
    ``max_steps`` counts as unfinished (``finished`` < ``episodes``) and is left out of the mean."""
    model = ACPathNet(net_cfg, 1, device, "torch")
    model.store.flat.data.copy_(flat.detach().to(model.store.flat.device, torch.float32))
    model.set_paths(np.asarray(expressed, np.float32)[None])
    model.task = task
    gen = torch.Generator(device=device).manual_seed(seed)
    kw = {} if env_id.startswith("CartPole") else dict(frameskip=frameskip, gray=gray)
    # on a GPU the env steps in its HIP kernel (bit-exact to the torch game, tests/test_envs.py / test_games_hip.py):
    # the torch Pong's per-sub-frame ops made a 7 K-step evaluation take 65 s
    backend = "hip" if torch.device(device).type == "cuda" else "torch"
    try:
        env = make(env_id, num_envs=episodes, device=device, seed=seed, backend=backend, **kw)
    except (NotImplementedError, ValueError, RuntimeError):
        env = make(env_id, num_envs=episodes, device=device, seed=seed, backend="torch", **kw)
    obs = env.reset()
    state = model.init_state(episodes)
    ret = torch.zeros(episodes, device=device)
    fin = torch.zeros(episodes, dtype=torch.bool, device=device)
    steps = 0
    for steps in range(1, max_steps + 1):
        logits, _, state = model.forward(obs, episodes, state)
        a = torch.multinomial(torch.softmax(logits.float(), -1), 1, generator=gen).reshape(-1)
        obs, _, d, info = env.step(a)
        d = d.bool()
        first = d & ~fin
        ret = torch.where(first, info["episode_return"].float(), ret)
        fin |= d
        if state is not None:
            keep = (~d).float()[:, None]
            state = (state[0] * keep, state[1] * keep)
        if steps % check_every == 0 and bool(fin.all()):
            break
    r = ret[fin].cpu().numpy().astype(np.float64)
    return {"mean": float(r.mean()) if r.size else float("nan"), "min": float(r.min()) if r.size else None,
            "max": float(r.max()) if r.size else None, "finished": int(r.size), "episodes": int(episodes),
            "steps": int(steps), "policy": "sampled", "seed": int(seed),
            "returns": [float(x) for x in r]}
