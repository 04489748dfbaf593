"""Where the rectangle rasteriser's time goes (csrc/preprocess.hip rects_push_kernel<true>): the frame-ring push of
every pixel game's scene at 2048 envs, banded vs the per-row walk over every rectangle, and with no rectangles at all
(background fill + resize + ring store only) -- a measurement split, not a shipped variant.  Interleaved rounds,
median us per launch.

    python scripts/diag/rects_phases.py [--envs 2048]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from pathnet_gym_amd.envs.atari_games import AlienVec, BreakoutVec, CentipedeVec, SpaceInvadersVec  # noqa: E402
from pathnet_gym_amd.ops import _lib  # noqa: E402
from pathnet_gym_amd.ops import envs as henv  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=6)
    a = ap.parse_args()
    lib = _lib.lib()
    out = {}
    for cls in (AlienVec, CentipedeVec, BreakoutVec, SpaceInvadersVec):
        g = cls(a.envs, device="cuda", seed=1, backend="hip")
        g.reset() if hasattr(g, "reset") else None
        N = a.envs
        act = torch.randint(0, g.num_actions, (N,), dtype=torch.int32, device="cuda")
        rw = torch.zeros(N, device="cuda")
        dn = torch.zeros(N, dtype=torch.uint8, device="cuda")
        ep = torch.zeros(N, device="cuda")
        frames = torch.zeros(N, 8, 160 * 120, dtype=torch.uint8, device="cuda")
        fc_in = torch.zeros(N, dtype=torch.uint8, device="cuda")
        fc_out = torch.zeros_like(fc_in)
        for _ in range(30):                       # a lived-in scene
            g._hip_run(act, None, rw, dn, ep)
        rects = g._rects
        empty = rects[:, :0].contiguous()
        arms = {
            "banded": lambda: (lib.rects_set_banded(2), henv.rects16_ring_push(rects, g._gray_tab, g._bg_gray, frames, 3, fc_in, fc_out, dn, g._tab32)),
            "walk_all": lambda: (lib.rects_set_banded(0), henv.rects16_ring_push(rects, g._gray_tab, g._bg_gray, frames, 3, fc_in, fc_out, dn, g._tab32)),
            "no_rects": lambda: (lib.rects_set_banded(2), henv.rects16_ring_push(empty, g._gray_tab[:0], g._bg_gray, frames, 3, fc_in, fc_out, dn, g._tab32)),
        }
        t = {k: [] for k in arms}
        for r in range(a.rounds):
            for k, fn in arms.items():
                fn()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.reps):
                    fn()
                e.record()
                torch.cuda.synchronize()
                t[k].append(s.elapsed_time(e) / a.reps * 1e3)
        lib.rects_set_banded(1)
        out[cls.id] = {"rects": int(rects.shape[1]), **{k: round(statistics.median(v), 1) for k, v in t.items()}}
        print(json.dumps({cls.id: out[cls.id]}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
