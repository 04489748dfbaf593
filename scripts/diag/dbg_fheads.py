"""Where do the fused and unfused last-layer + heads rollouts diverge (tests/test_x3_engine.py fused heads test)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from pathnet_gym_amd.config import preset
from pathnet_gym_amd.algo.trainer import PathNetTrainer

runs = []
for fuse in ("0", "1"):
    os.environ["PATHNET_X3_FUSE_HEADS"] = fuse
    cfg = preset("pong")
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 4, 32, 5
    cfg.compute_dtype = "fp32x"
    cfg.frame_ring = True
    cfg.use_graph = False
    cfg.ga.backend = "device"
    cfg.a2c.lr = 0.0
    tr = PathNetTrainer(cfg, device="cuda")
    e = tr.engine
    tr.env.max_episode_steps = 7
    snaps = []
    for _ in range(4):
        tr.update()
        torch.cuda.synchronize()
        snaps.append({"feat": e.acts[-1].clone(), "fc1": e.acts[-2].clone(), "c1": e.acts[0].clone(),
                      "bits": e.bits[-1].clone(), "logits": e.logits.clone(), "values": e.values.clone(),
                      "actions": e.actions.clone(), "w": tr.model.store.flat.detach().clone(),
                      "act_idx": tr.model.act_idx.clone(), "frames": e.frames.clone(), "gen": tr.pop.generation})
    runs.append(snaps)
for u, (a, b) in enumerate(zip(*runs)):
    for k in a:
        if k == "gen":
            print(u, "gen", a[k], b[k]); continue
        x, y = a[k], b[k]
        if torch.equal(x, y):
            print(u, k, "equal"); continue
        d = (x.float() - y.float()).abs()
        nz = (d > 0).nonzero()
        print(u, k, "max", float(d.max()), "n", nz.shape[0], "first idx", nz[:3].tolist())
