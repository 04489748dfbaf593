#!/usr/bin/env python3
"""Calibrate the synthetic games' solve thresholds from a random policy and a scripted expert.

For every synthetic game this plays N envs (torch backend, CPU or GPU) with
* ``random``: uniform actions over the game's action set;
* ``expert``: a hand-written controller that reads the game STATE (not pixels) -- Pong/Breakout track the ball,
  SpaceInvaders fires under the nearest live column and side-steps bombs, Alien/MsPacman follow a breadth-first
  distance field to the nearest egg around the aliens, Centipede stays under the lowest segment and fires;
and records the mean episode return of each.  The threshold written to ``pathnet_gym_amd/envs/thresholds.json`` is

    threshold = random + FRACTION * (expert - random)

so "solved" means most of the way from chance to a competent scripted player.  Pong keeps the ALE convention 18
(the bench metric) when that is above its calibrated value.

    python scripts/calibrate_thresholds.py --envs 64 --out pathnet_gym_amd/envs/thresholds.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

FRACTION = 0.75


# ---------------------------------------------------------------------------------------------------------------
# experts (state -> action); every one is vectorised over envs
# ---------------------------------------------------------------------------------------------------------------
def pong_expert(env):
    from pathnet_gym_amd.envs import pong as P
    st = env.state
    centre = st[:, P.PY] + (P.PADDLE_H * P.U) // 2
    ball = st[:, P.BY] + (P.BALL_H * P.U) // 2
    mid = torch.full_like(ball, (P.TOP + P.BOTTOM) // 2 * P.U)
    target = torch.where(st[:, P.VX] > 0, ball, mid)
    a = torch.zeros_like(ball)
    a = torch.where(target < centre - P.U * 2, torch.full_like(a, 2), a)      # up
    a = torch.where(target > centre + P.U * 2, torch.full_like(a, 3), a)      # down
    return a


def breakout_expert(env):
    U = env.U
    centre = env.px + (env.PADDLE_W // 2) * U
    a = torch.ones_like(env.px)                                                # FIRE (serve)
    follow = env.inplay
    a = torch.where(follow, torch.zeros_like(a), a)
    a = torch.where(follow & (env.bx > centre + 2 * U), torch.full_like(a, 2), a)
    a = torch.where(follow & (env.bx < centre - 2 * U), torch.full_like(a, 3), a)
    return a


def invaders_expert(env):
    N, d = env.num_envs, env.device
    # the formation lands when its LOWEST live row reaches the ground: clear the lowest row first
    rows = torch.arange(env.AR, device=d)[None, :, None]
    lowest = torch.where(env.alive, rows, -1).flatten(1).max(1).values
    alive_cols = (env.alive & (rows == lowest[:, None, None])).any(1)        # [N, AC]
    cx = env.fx[:, None] + 16 * torch.arange(env.AC, device=d)[None] + 4      # column centres
    gun = env.px + 3
    dist = torch.where(alive_cols, (cx - gun[:, None]).abs(), torch.full_like(cx, 1 << 20))
    target = cx.gather(1, dist.argmin(1, keepdim=True)).squeeze(1)
    a = torch.ones(N, dtype=torch.int64, device=d)                             # FIRE
    a = torch.where(target > gun + 1, torch.full_like(a, 4), a)                # RIGHTFIRE
    a = torch.where(target < gun - 1, torch.full_like(a, 5), a)                # LEFTFIRE
    # a falling bomb within reach: keep moving away from its column until it has passed (bombs fall 8 px and
    # the gun moves 8 px per agent step)
    danger = env.bomb & (env.byp > 90) & ((env.bxp - gun).abs() < 14)
    go_right = (env.bxp <= gun) & (env.px < 126) | (env.px <= 26)
    a = torch.where(danger & go_right, torch.full_like(a, 4), a)
    a = torch.where(danger & ~go_right, torch.full_like(a, 5), a)
    return a


def alien_expert(env):
    """Distance field (multi-source BFS) to the nearest egg on free cells that are not next to an alien; step to
    the neighbour with the smallest distance (or away from the nearest alien when boxed in)."""
    N, d = env.num_envs, env.device
    H, W = env.H, env.W
    free = (~env.walls)[None].expand(N, H, W).clone()
    yy = torch.arange(H, device=d)[None, :, None]
    xx = torch.arange(W, device=d)[None, None, :]
    danger = torch.zeros(N, H, W, dtype=torch.bool, device=d)
    for k in range(env.NA):
        dist = (yy - env.ay[:, k, None, None]).abs() + (xx - env.ax[:, k, None, None]).abs()
        danger |= dist <= 1
    ok = free & ~danger
    INF = 1 << 16
    dist = torch.where(env.dots & ok, 0, INF)
    for _ in range(H * W // 2):
        pad = torch.nn.functional.pad(dist, (1, 1, 1, 1), value=INF)
        nb = torch.stack([pad[:, :-2, 1:-1], pad[:, 2:, 1:-1], pad[:, 1:-1, :-2], pad[:, 1:-1, 2:]]).min(0).values
        new = torch.where(ok, torch.minimum(dist, nb + 1), dist)
        if torch.equal(new, dist):
            break
        dist = new
    ar = torch.arange(N, device=d)
    best = torch.full((N,), INF + 1, dtype=torch.int64, device=d)
    act = torch.zeros(N, dtype=torch.int64, device=d)
    # direction index j (1 up, 2 right, 3 left, 4 down) is ALE action j + 1
    for j in range(1, 5):
        cy = (env.py + env.dy[j]).clamp(0, H - 1)
        cx = (env.px + env.dx[j]).clamp(0, W - 1)
        dj = torch.where(ok[ar, cy, cx], dist[ar, cy, cx], torch.full_like(best, INF + 1))
        better = dj < best
        best = torch.where(better, dj, best)
        act = torch.where(better, torch.full_like(act, j + 1), act)
    # boxed in: step to the free neighbour farthest from the nearest alien
    stuck = best >= INF
    far = torch.full((N,), -1, dtype=torch.int64, device=d)
    for j in range(1, 5):
        cy = (env.py + env.dy[j]).clamp(0, H - 1)
        cx = (env.px + env.dx[j]).clamp(0, W - 1)
        md = ((env.ay - cy[:, None]).abs() + (env.ax - cx[:, None]).abs()).min(1).values
        md = torch.where(free[ar, cy, cx], md, torch.full_like(md, -1))
        better = stuck & (md > far)
        far = torch.where(better, md, far)
        act = torch.where(better, torch.full_like(act, j + 1), act)
    return act


def centipede_expert(env):
    """Fire continuously (clearing the mushrooms overhead slows the centipede's descent) and stand where the
    nearest segment of the lowest row will be when the shot arrives (shots rise 6 px per sub-frame, segments move
    one 10-px column every 3 sub-frames)."""
    N, d = env.num_envs, env.device
    low = torch.where(env.salive, env.sy, torch.full_like(env.sy, -1))
    lowest = low.max(1, keepdim=True).values
    gun = env.px + 2
    cand = env.salive & (env.sy == lowest)
    travel = (180 - (20 + 8 * env.sy)).clamp(min=0) // 6                       # sub-frames to reach the row
    lead = (env.sx + env.sdir * (travel // 3)).clamp(0, env.GW - 1)
    segx = lead * 10 + 5
    dist = torch.where(cand, (segx - gun[:, None]).abs(), torch.full_like(segx, 1 << 20))
    target = segx.gather(1, dist.argmin(1, keepdim=True)).squeeze(1)
    a = torch.ones(N, dtype=torch.int64, device=d)                             # FIRE
    a = torch.where(target > gun + 2, torch.full_like(a, 12), a)               # RIGHT + FIRE
    a = torch.where(target < gun - 2, torch.full_like(a, 13), a)               # LEFT + FIRE
    return a


EXPERTS = {"Pong": pong_expert, "Breakout": breakout_expert, "SpaceInvaders": invaders_expert,
           "Alien": alien_expert, "MsPacman": alien_expert, "Centipede": centipede_expert}


def play(game: str, policy: str, n: int, episodes: int, max_steps: int, device, seed: int = 7):
    from pathnet_gym_amd.envs.registry import make
    env = make(game, num_envs=n, device=device, seed=seed, backend="torch")
    env.reset()
    g = torch.Generator(device="cpu").manual_seed(seed)
    rets = [[] for _ in range(n)]
    steps = 0
    pixels = game == "Pong"        # the other games step physics only (no render needed for scoring)
    while steps < max_steps and min(len(r) for r in rets) < episodes:
        if policy == "random":
            a = torch.randint(0, env.num_actions, (n,), generator=g).to(device)
        else:
            a = EXPERTS[game](env)
        if pixels:
            _, _, done, info = env.step(a)
            ep = info["episode_return"]
        else:
            _, done, ep = env._advance(a)
        steps += 1
        for i in torch.nonzero(done).flatten().tolist():
            rets[i].append(float(ep[i]))
    flat = [x for r in rets for x in r[:episodes]]
    unfinished = sum(1 for r in rets if not r)
    return {"mean_return": sum(flat) / max(1, len(flat)), "episodes": len(flat), "agent_steps": steps,
            "envs_without_episode": unfinished}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", default="Pong,Breakout,SpaceInvaders,Alien,MsPacman,Centipede")
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--episodes", type=int, default=2)
    ap.add_argument("--max-steps", type=int, default=27000)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from pathnet_gym_amd.envs.registry import REAL_ATARI_THRESHOLDS
    res = {}
    for game in [x.strip() for x in args.games.split(",")]:
        t0 = time.time()
        r = play(game, "random", args.envs, args.episodes, args.max_steps, args.device)
        e = play(game, "expert", args.envs, args.episodes, args.max_steps, args.device)
        thr = r["mean_return"] + FRACTION * (e["mean_return"] - r["mean_return"])
        if game == "Pong":
            thr = max(thr, REAL_ATARI_THRESHOLDS["Pong"])
        thr = float(round(thr, 1))
        res[game] = {"threshold": thr, "random": r, "expert": e, "fraction": FRACTION,
                     "seconds": round(time.time() - t0, 1)}
        print(json.dumps({game: res[game]}), flush=True)
    if args.out:
        doc = {"rule": f"threshold = random + {FRACTION} * (expert - random) (Pong: max with the ALE 18)",
               "source": "scripts/calibrate_thresholds.py", "envs": args.envs, "episodes_per_env": args.episodes,
               "games": res}
        with open(args.out, "w") as f:
            json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
