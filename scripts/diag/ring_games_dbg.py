"""Debug: HIP game frame-ring plane vs packed stack channel 3 after one step."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from pathnet_gym_amd.envs.atari_games import GAMES
N = 8
for name in ("Breakout", "SpaceInvaders"):
    ep = GAMES[name](N, device="cuda", seed=7, backend="hip")
    er = GAMES[name](N, device="cuda", seed=7, backend="hip")
    o0 = ep.reset(); o1 = er.reset()
    print(name, "reset equal", torch.equal(o0, o1), "o0 nonzero", int((o0 != 0).sum()), "R", er._rects.shape)
    frames = torch.zeros(N, 8, 160 * 120, dtype=torch.uint8, device="cuda")
    fc = torch.zeros(2, N, dtype=torch.uint8, device="cuda")
    rw, dn, eret = torch.zeros(N, device="cuda"), torch.zeros(N, dtype=torch.uint8, device="cuda"), torch.zeros(N, device="cuda")
    a = torch.zeros(N, dtype=torch.int64, device="cuda")
    obs, r, d, _ = ep.step(a)
    er.step_ring_into(a.to(torch.int32), frames, 4, fc[0], fc[1], rw, dn, eret)
    torch.cuda.synchronize()
    new_p = obs[..., 3].reshape(N, -1)
    new_r = frames[:, 4]
    mm = (new_p != new_r)
    print(" rects equal", torch.equal(ep._rects, er._rects), "mismatch", int(mm.sum()), "of", mm.numel(),
          "packed nz", int((new_p != 0).sum()), "ring nz", int((new_r != 0).sum()), "fc1", fc[1].tolist(), "done", dn.tolist())
    idx = mm[0].nonzero()[:8].flatten().tolist()
    print(" env0 first mismatches", [(i // 120, i % 120, int(new_p[0, i]), int(new_r[0, i])) for i in idx])
