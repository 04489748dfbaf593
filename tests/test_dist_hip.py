"""The multi-rank path that ships, on one MI355X: 2 gloo ranks sharing the GPU.

HIP engine + device GA + pipelined ``exchange_async`` + hipGraphs + ``check_every=1`` (replica
digests all-gathered after every update).  Checks, on both ranks:
* the all-reduced gradient equals the sum of the per-rank gradients on every packed range;
* the device genotype table equals the host mirror of the device GA;
* after a task switch freezes modules, the active-path plan is sparse (frozen modules excluded) and
  ``comm.bytes_last`` is below the dense payload.
RCCL itself needs one GPU per rank, so the 8-GPU path runs only on the driver's node; this test runs the
same code over gloo (``PATHNET_DIST_BACKEND=gloo``).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), PATHNET_DIST_BACKEND="gloo")
    torch.set_num_threads(2)
    try:
        import torch.distributed as dist
        from pathnet_gym_amd.algo.trainer import PathNetTrainer
        from pathnet_gym_amd.config import preset
        from pathnet_gym_amd.parallel.dist import init_distributed
        ctx = init_distributed()
        cfg = preset("pong")
        cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 4, 16, 4
        cfg.ga.backend = "device"
        cfg.ga.concurrent_tournaments = 1
        cfg.net.N = 2                         # sparse unions at this small population size
        cfg.check_every = 1
        cfg.tasks = ["Pong", "Pong"]
        tr = PathNetTrainer(cfg, device=ctx.device, ctx=ctx)
        assert tr.pipelined and tr.engine.use_graph and not tr.comm.force_dense
        out = {"grad_checks": 0, "grad_ok": True}
        comm = tr.comm
        orig = comm._reduce

        def checked(grad, fit, cnt):
            local = grad.detach().cpu()
            n = orig(grad, fit, cnt)
            torch.cuda.synchronize()
            parts = [torch.zeros_like(local) for _ in range(world)]
            dist.all_gather(parts, local)
            tot = parts[0] + parts[1]
            red = grad.detach().cpu()
            for s, e in comm.ranges:
                if not torch.equal(red[s:e], tot[s:e]):
                    out["grad_ok"] = False
            out["grad_checks"] += 1
            return n
        comm._reduce = checked
        for _ in range(12):
            tr.update()
        tr.flush()
        torch.cuda.synchronize()
        g = tr.engine.ga_dev
        out["geno_match"] = bool(np.array_equal(g["geno"].cpu().numpy(), tr.pop.genotypes.astype(np.uint8)))
        out["dense_bytes"] = (tr.model.store.layout.numel + comm.P_total + comm.NCOUNTERS) * 4
        out["bytes_task0"] = comm.bytes_last
        tr.end_task()
        tr._start_task(1)
        frozen = tr.pop.frozen > 0.5
        for _ in range(8):
            tr.update()
        tr.flush()
        torch.cuda.synchronize()
        out["bytes_task1"] = comm.bytes_last
        out["dense_task1"] = comm.dense
        lay = tr.model.store.layout
        out["frozen_excluded"] = all(not (s < lay.module_range(l, j)[1] and lay.module_range(l, j)[0] < e)
                                     for s, e in comm.ranges for l in range(cfg.net.L) for j in range(cfg.net.M)
                                     if frozen[l, j])
        g = tr.engine.ga_dev
        out["geno_match_task1"] = bool(np.array_equal(g["geno"].cpu().numpy(), tr.pop.genotypes.astype(np.uint8)))
        out["flat"] = tr.model.store.flat.detach().cpu().numpy().copy()
        out["gen"] = tr.pop.generation
        q.put((rank, out))
        ctx.destroy()
    except Exception:   # pragma: no cover
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))


def test_two_gloo_ranks_on_one_gpu_hip_engine_device_ga_pipelined(hip_lib):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(60)
    for r in range(2):
        assert "error" not in res[r], res[r].get("error")
    a, b = res[0], res[1]
    for o in (a, b):
        assert o["grad_checks"] == 20 and o["grad_ok"]
        assert o["geno_match"] and o["geno_match_task1"]
        assert not o["dense_task1"] and o["frozen_excluded"]
        assert o["bytes_task1"] < o["dense_bytes"]
    assert np.array_equal(a["flat"], b["flat"]) and a["gen"] == b["gen"]
