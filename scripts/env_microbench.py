#!/usr/bin/env python3
"""Micro-benchmark of the on-device Pong env step kernels (packed stack push vs frame ring).

    python scripts/env_microbench.py [--envs 2048] [--iters 200]
Prints one JSON line per variant with the mean kernel time (us) measured with HIP events.
"""
from __future__ import annotations

import argparse
import json

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=200)
    args = ap.parse_args()
    from pathnet_gym_amd import _build
    _build.build()
    from pathnet_gym_amd.envs.pong import PongVec
    from pathnet_gym_amd.ops import envs as henv
    dev = "cuda:0"
    B = args.envs
    env = PongVec(B, device=dev, backend="hip", seed=3)
    env.reset()
    acts = torch.randint(0, 6, (B,), dtype=torch.int32, device=dev)
    r = torch.empty(B, device=dev)
    d = torch.empty(B, dtype=torch.uint8, device=dev)
    e = torch.empty(B, device=dev)
    stack_a = env.obs.reshape(B, -1).contiguous()
    stack_b = torch.empty_like(stack_a)
    frames = torch.zeros(B, 24, 160 * 120, dtype=torch.uint8, device=dev)
    fc = torch.zeros(2, B, dtype=torch.uint8, device=dev)

    def timeit(fn):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(args.iters):
            fn()
        t.record()
        torch.cuda.synchronize()
        return s.elapsed_time(t) * 1e3 / args.iters

    base_fs = env.frameskip
    for fs in (base_fs, 0):
        env.frameskip = fs
        us_p = timeit(lambda: henv.pong_step_into(env, acts, stack_a, stack_b, r, d, e))
        us_r = timeit(lambda: henv.pong_step_ring_into(env, acts, frames, 5, fc[0], fc[1], r, d, e))
        print(json.dumps({"envs": B, "frameskip": fs, "packed_us": round(us_p, 2), "ring_us": round(us_r, 2)}))
    env.frameskip = base_fs


if __name__ == "__main__":
    main()
