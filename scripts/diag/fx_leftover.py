"""Deterministic fp32x: which accumulator entries stay non-zero after a backward's flush (layer / segment map)."""
import sys
import torch
sys.path.insert(0, ".")
from pathnet_gym_amd import _build
_build.build()
from pathnet_gym_amd.config import preset
from pathnet_gym_amd.algo.trainer import PathNetTrainer

for ring in (False, True):
    cfg = preset("pong")
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 3, 16, 4
    cfg.use_graph = False
    cfg.compute_dtype = "fp32x"
    cfg.frame_ring = ring
    cfg.deterministic = True
    tr = PathNetTrainer(cfg, device="cuda")
    eng = tr.engine
    tr.env.max_episode_steps = 5
    tr.update()
    torch.cuda.synchronize()
    fx = tr.model.hip._fxbuf
    print("ring", ring, "after update: nonzero", int((fx != 0).sum()), "guard", int(fx[0]))
    eng._rollout_backward_body()
    torch.cuda.synchronize()
    nz = torch.nonzero(fx[1:]).flatten()
    print("after body: nonzero", nz.numel(), "guard", int(fx[0]))
    if nz.numel():
        idx = nz.cpu().numpy()
        for s in tr.model.store.layout.segments:
            m = ((idx >= s.offset) & (idx < s.offset + s.numel)).sum()
            if m:
                print("  segment", s.name, "layer", s.layer, "module", s.module, "left", int(m), "of", s.numel,
                      "vals", fx[1:][s.offset:s.offset + s.numel][fx[1:][s.offset:s.offset + s.numel] != 0][:4].tolist())
