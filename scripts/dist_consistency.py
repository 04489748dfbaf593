"""Multi-rank consistency check on GPU: after K updates every rank must hold identical weights,
RMSProp slots and GA state (run under torch.distributed.run)."""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

from pathnet_gym_amd.algo.trainer import PathNetTrainer
from pathnet_gym_amd.config import preset
from pathnet_gym_amd.parallel.dist import init_distributed


def digest(*arrs):
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def main():
    ctx = init_distributed()
    cfg = preset("pong")
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 8, 16, 5
    cfg.ga.concurrent_tournaments = 4
    tr = PathNetTrainer(cfg, device=ctx.device, ctx=ctx)
    for i in range(6):
        tr.update()
    torch.cuda.synchronize()
    d = digest(tr.model.store.flat.detach().cpu().numpy(), tr.opt.ms.cpu().numpy(), tr.pop.genotypes,
               np.array([tr.global_step, tr.pop.generation]))
    t = torch.tensor([int(d[:12], 16)], dtype=torch.float64, device=ctx.device)
    mx, mn = t.clone(), t.clone()
    torch.distributed.all_reduce(mx, op=torch.distributed.ReduceOp.MAX)
    torch.distributed.all_reduce(mn, op=torch.distributed.ReduceOp.MIN)
    ok = bool(mx.item() == mn.item())
    print(f"rank {ctx.rank}: digest {d[:16]} steps {tr.global_step} gens {tr.pop.generation} consistent={ok}", flush=True)
    ctx.destroy()
    if not ok:
        raise SystemExit(1)


if __name__ == "__main__":
    main()
