"""Multi-process (gloo, world_size 2) tests: the fused all-reduce and replicated GA.

Each rank runs its own PathNetTrainer (CPU, torch backend) on its half of the
population.  After every update all ranks must hold bit-identical weights,
optimizer slots and GA state, and the all-reduced gradient must equal the
sum of the per-rank gradients.  Uses 127.0.0.1 rendezvous.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mode, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    try:
        from pathnet_gym_amd.algo.trainer import PathNetTrainer
        from pathnet_gym_amd.config import preset
        from pathnet_gym_amd.parallel.dist import init_distributed
        ctx = init_distributed(device="cpu", backend="gloo")
        cfg = preset("cartpole-cpu")
        cfg.paths, cfg.envs_per_path = 3, 4
        cfg.ga.B = 2
        cfg.ga.concurrent_tournaments = 2
        cfg.ga_sync = "fused" if mode == "diverge" else mode
        cfg.check_every = 2
        tr = PathNetTrainer(cfg, ctx=ctx)
        out = {}
        if mode == "diverge":
            from pathnet_gym_amd.runtime.consistency import DivergenceError
            tr.update()
            if rank == 1:
                with torch.no_grad():
                    tr.model.store.flat[7] += 1e-3       # a replica silently drifts
            try:
                tr.update()
                out["raised"] = False
            except DivergenceError as e:
                out["raised"] = "[1]" in str(e)
            q.put((rank, out))
            ctx.destroy()
            return
        if mode == "fused":
            # all-reduced grad == sum of local grads
            g, c, _ = tr.rollout_and_backward()
            local = g.clone()
            tot = torch.zeros_like(local)
            dist.all_reduce(local.clone(), op=dist.ReduceOp.SUM)
            gl = [torch.zeros_like(local) for _ in range(world)]
            dist.all_gather(gl, local)
            tot = sum(gl)
            tr.comm.exchange(g, tr.fitness_local, c)
            out["grad_ok"] = bool(torch.allclose(g, tot, atol=1e-5))
        for _ in range(6):
            tr.update()
        out["flat"] = tr.model.store.flat.detach().numpy().copy()
        out["ms"] = tr.opt.ms.numpy().copy()
        out["geno"] = tr.pop.genotypes.copy()
        out["gen"] = tr.pop.generation
        out["step"] = tr.global_step
        q.put((rank, out))
        ctx.destroy()
    except Exception as e:   # pragma: no cover
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))


@pytest.mark.parametrize("mode", ["fused", "gather_bcast"])
def test_two_ranks_stay_in_lockstep(mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, mode, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(60)
    for r in range(2):
        assert "error" not in res[r], res[r].get("error")
    a, b = res[0], res[1]
    assert np.array_equal(a["flat"], b["flat"])
    assert np.array_equal(a["ms"], b["ms"])
    assert np.array_equal(a["geno"], b["geno"])
    assert a["gen"] == b["gen"] and a["step"] == b["step"]
    assert a["step"] == 6 * 2 * 3 * 4 * 5
    if mode == "fused":
        assert a["grad_ok"] and b["grad_ok"]


def test_replica_divergence_is_detected_on_every_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, "diverge", q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(60)
    for r in range(2):
        assert "error" not in res[r], res[r].get("error")
        assert res[r]["raised"] is True


# ---------------------------------------------------------------------------------------------------------------
# strong scaling (TrainConfig.paths_total): a fixed population split over the ranks computes the one-process run
# ---------------------------------------------------------------------------------------------------------------
def _strong_cfg():
    from pathnet_gym_amd.config import preset
    cfg = preset("cartpole-cpu")
    cfg.paths_total, cfg.envs_per_path = 8, 4
    cfg.ga.B = 2
    cfg.ga.concurrent_tournaments = 2
    return cfg


def _strong_run(tr, updates=8):
    hist = []
    for _ in range(updates):
        st = tr.update()
        hist.append((st.episodes, st.tournaments, tr.pop.generation, tr.global_step))
    return {"flat": tr.model.store.flat.detach().numpy().copy(), "ms": tr.opt.ms.numpy().copy(),
            "geno": tr.pop.genotypes.copy(), "fit": tr.pop.fitness.copy(), "gen": tr.pop.generation,
            "step": tr.global_step, "hist": hist, "P": tr.P}


def _strong_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    try:
        from pathnet_gym_amd.algo.trainer import PathNetTrainer
        from pathnet_gym_amd.parallel.dist import init_distributed
        ctx = init_distributed(device="cpu", backend="gloo")
        tr = PathNetTrainer(_strong_cfg(), ctx=ctx)
        out = _strong_run(tr)
        q.put((rank, out))
        ctx.destroy()
    except Exception:   # pragma: no cover
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))


def test_strong_scaling_four_ranks_reproduce_one_process():
    """4 gloo ranks x 2 paths (paths_total = 8) vs one process with the 8 paths: same env streams, same sampled
    actions, same episodes, the same GA decisions and genotypes; the weights differ only by the summation order of
    the gradient (per-rank partial sums + all-reduce vs one backward)."""
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    torch.set_num_threads(1)
    one = _strong_run(PathNetTrainer(_strong_cfg()))
    assert one["P"] == 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_strong_worker, args=(r, 4, port, q)) for r in range(4)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(60)
    for r in range(4):
        assert "error" not in res[r], res[r].get("error")
        assert res[r]["P"] == 2
    four = res[0]
    assert four["hist"] == one["hist"]                       # episodes, tournaments, generations, frames per update
    assert four["gen"] == one["gen"] > 0 and four["step"] == one["step"]
    assert np.array_equal(four["geno"], one["geno"])
    assert np.array_equal(four["fit"], one["fit"])
    np.testing.assert_allclose(four["flat"], one["flat"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(four["ms"], one["ms"], rtol=1e-4, atol=1e-6)
    for r in range(1, 4):                                      # replicas stay bit-identical across ranks
        assert np.array_equal(res[r]["flat"], four["flat"])


def test_single_rank_exchange_packs_the_report():
    """One rank: fitness, counters and the report parts are packed by one cat and read back by one copy
    (parallel/comm.py exchange_async); the reduced views the device GA reads hold the fitness and counters; a tensor
    report and no report keep working."""
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    from pathnet_gym_amd.config import preset
    cfg = preset("cartpole-cpu")
    cfg.paths, cfg.envs_per_path = 3, 4
    tr = PathNetTrainer(cfg, device="cpu")
    comm = tr.comm
    assert not comm.ctx.enabled
    P = comm.P_total
    fit = torch.arange(P, dtype=torch.float32) + 0.5
    cnt = torch.tensor([1.0, 2.0, 3.0, 4.0])
    f, c, e = comm.collect(comm.exchange_async(None, fit, cnt, extra=(torch.tensor([5.0, 6.0, 7.0, 8.0]),
                                                                      torch.tensor([9.0]))))
    assert np.array_equal(f, fit.numpy()) and np.array_equal(c, cnt.numpy())
    assert np.array_equal(e, np.array([5.0, 6.0, 7.0, 8.0, 9.0], dtype=np.float32))
    assert torch.equal(comm.fit_reduced, fit) and torch.equal(comm.cnt_reduced, cnt)
    f, c, e = comm.collect(comm.exchange_async(None, fit, cnt, extra=torch.tensor([1.0, 2.0])))
    assert np.array_equal(e, np.array([1.0, 2.0], dtype=np.float32)) and np.array_equal(c, cnt.numpy())
    f, c, e = comm.collect(comm.exchange_async(None, fit, cnt))
    assert e is None and np.array_equal(f, fit.numpy())
