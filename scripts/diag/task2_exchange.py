"""Time the update on a forced one-rank RCCL group (PATHNET_DIST_FORCE=1: every collective of the multi-GPU path runs)
in task 1 (static all-reduce plan: every trainable module) and in task 2 after the freeze (frozen modules leave the
plan), with the static plan and with the EXACT plan (only the modules the running population expresses, read back
from the device GA after every optimizer step: trainer._plan_exchange forced via static_plan_min_density > 1).
Medians of --windows windows of --steps updates; the same shapes without a group for reference.

    PATHNET_DIST_FORCE=1 python scripts/diag/task2_exchange.py --paths 8
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--paths", type=int, default=8)
    ap.add_argument("--envs", type=int, default=32)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--windows", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=5)
    args = ap.parse_args()
    import torch
    from pathnet_gym_amd import _build
    _build.build()
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    from pathnet_gym_amd.config import preset
    from pathnet_gym_amd.parallel.dist import init_distributed
    ctx = init_distributed()
    cfg = preset("pong")
    cfg.tasks = ["Pong", "Breakout"]
    cfg.paths, cfg.envs_per_path = args.paths, args.envs
    cfg.backend, cfg.compute_dtype, cfg.frame_ring = "hip", "fp32x", True
    cfg.ga.backend = "device"
    cfg.ga.concurrent_tournaments = max(1, args.paths // 16)
    tr = PathNetTrainer(cfg, device=ctx.device, ctx=ctx)

    def windows():
        for _ in range(args.warmup):
            tr.update()
        tr.flush()
        out = []
        for _ in range(args.windows):
            torch.cuda.synchronize()
            ctx.barrier()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                tr.update()
            tr.flush()
            torch.cuda.synchronize()
            out.append((time.perf_counter() - t0) / args.steps * 1e3)
        return {"median_ms": round(statistics.median(out), 3), "windows_ms": [round(x, 3) for x in out],
                "plan": getattr(tr, "plan_mode", "none"), "reduced_grad_numel": int(getattr(tr.comm, "ngrad", -1)),
                "plans": int(getattr(tr.comm, "plans", 0))}

    rec = {"paths": args.paths, "envs": args.envs, "world": ctx.world, "forced_group": bool(ctx.enabled),
           "backend": ctx.backend}
    rec["task1_static"] = windows()
    tr.end_task()
    tr._start_task(1)
    rec["frozen_modules"] = int((tr.pop.frozen > 0.5).sum())
    rec["task2_static"] = windows()
    tr.static_plan_min_density = 1.01         # the exact plan: only the modules the population expresses
    rec["task2_exact"] = windows()
    if ctx.is_main:
        print(json.dumps(rec), flush=True)
    ctx.destroy()


if __name__ == "__main__":
    main()
