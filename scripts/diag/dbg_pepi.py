"""Where does the pipelined-epilogue band forward (X3_C1_EPIBF=2) differ from the branch-free one (=1)?"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from pathnet_gym_amd.config import preset
from pathnet_gym_amd.algo.trainer import PathNetTrainer
from pathnet_gym_amd.ops import _lib

cfg = preset("pong")
cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 3, 16, 4
cfg.compute_dtype = "fp32x"
cfg.frame_ring = True
cfg.use_graph = False
tr = PathNetTrainer(cfg, device="cuda")
tr.update(); tr.flush(); torch.cuda.synchronize()
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from test_x3_engine import masks_with_edges
tr.model.set_paths(masks_with_edges(3, cfg.net.L, cfg.net.M, cfg.net.N, seed=2))
e, hp, lib = tr.engine, tr.model.hip, _lib.lib()
outs = []
for v in (1, 2):
    lib.fast_conv_set_x3_c1_epibf(v)
    e.acts[0].zero_(); e.bits[0].zero_()
    hp.ring_fwd(e.frames, e.fc, e.acts[0], e.bits[0], e.P, e.E, 1, 0, e.bits_rows[0])
    torch.cuda.synchronize()
    outs.append((e.acts[0].clone(), e.bits[0].clone()))
lib.fast_conv_set_x3_c1_epibf(0)
print("per-path first-layer counts", tr.model.act_cnt[:, 0].tolist())
a1, a2 = outs[0][0][0].view(torch.int16).reshape(e.B, 39 * 29, 8), outs[1][0][0].view(torch.int16).reshape(e.B, 39 * 29, 8)
d = (a1 != a2).any(-1)              # [B, positions]
print("act cnt", hp.model.act_cnt[:, 0].tolist())
print("differing (sample, position) pairs:", int(d.sum()), "of", d.numel())
rows = d.nonzero()
if rows.shape[0]:
    s = rows[:, 0]; pos = rows[:, 1]
    print("samples:", sorted(set(s.tolist()))[:20])
    band = (pos // 29) // 8
    print("bands:", sorted(set(band.tolist())))
    print("first:", rows[:10].tolist())
    print("zero in epibf2 at those:", bool((a2[d] == 0).all()))
b1, b2 = outs[0][1], outs[1][1]
print("bits differ:", int((b1 != b2).sum()))
