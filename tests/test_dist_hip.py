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
        cfg.overlap_allreduce = False         # the single-bucket exchange (the split one: tests below)
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
            inside = torch.zeros(local.numel(), dtype=torch.bool)
            for s, e in comm.ranges:
                inside[s:e] = True
                if not torch.equal(red[s:e], tot[s:e]):
                    out["grad_ok"] = False
            # outside the plan: untouched by the reduce, and zero unless the module is frozen (a frozen module on a
            # path still gets a local gradient that the optimizer discards); a plan lagging the rollout fails here
            if not torch.equal(red[~inside], local[~inside]):
                out["grad_ok"] = False
            frozen_mask = torch.zeros(local.numel(), dtype=torch.bool)
            fz = tr.pop.frozen > 0.5
            lay = tr.model.store.layout
            for l in range(cfg.net.L):
                for j in range(cfg.net.M):
                    if fz[l, j]:
                        s, e = lay.module_range(l, j)
                        frozen_mask[s:e] = True
            if torch.count_nonzero(local[~inside & ~frozen_mask]) != 0:
                out["grad_ok"] = False
                out["stray"] = int(torch.count_nonzero(local[~inside & ~frozen_mask]))
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


# ---------------------------------------------------------------------------------------------------------------
# overlapped all-reduce (TrainConfig.overlap_allreduce) and 4 ranks with tournaments firing
# ---------------------------------------------------------------------------------------------------------------
def _overlap_worker(rank, world, port, q, updates, trace_path, dtype="fp32", preset_name="pong", density=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), PATHNET_DIST_BACKEND="gloo")
    torch.set_num_threads(2)
    try:
        from pathnet_gym_amd.algo.trainer import PathNetTrainer
        from pathnet_gym_amd.config import preset
        from pathnet_gym_amd.parallel.dist import init_distributed
        ctx = init_distributed()
        out = {}
        for mode in ("overlap", "serial"):
            cfg = preset(preset_name)
            cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 4, 16, 4
            cfg.ga.backend = "device"
            cfg.ga.concurrent_tournaments = 2
            cfg.ga.fitness_window = 2           # small window: tournaments fire during the run
            cfg.net.N = 2
            # fp32: fixed-order reductions, bit-reproducible, so the modes compare bitwise; fp32x (the bench engine:
            # frame ring, float atomics in the weight gradients) compares to its budget
            cfg.compute_dtype = dtype
            cfg.frame_ring = dtype == "fp32x"
            cfg.overlap_allreduce = mode == "overlap"
            tr = PathNetTrainer(cfg, device=ctx.device, ctx=ctx)
            if density is not None:
                tr.static_plan_min_density = density      # 0: always the static plan; > 1: always the exact union
            tr.env.max_episode_steps = 6
            assert tr.engine.split == (mode == "overlap")
            if mode == "overlap":
                tr.comm.overlap_log = []
            for _ in range(updates):
                tr.update()
            tr.flush()
            torch.cuda.synchronize()
            out[mode] = dict(flat=tr.model.store.flat.detach().cpu().numpy().copy(), gen=tr.pop.generation,
                             geno=tr.pop.genotypes.copy(), ms=tr.opt.ms.detach().cpu().numpy().copy(),
                             plan_mode=getattr(tr, "plan_mode", None), lstm=bool(tr.engine.lstm_hip))
            if mode == "overlap":
                log = tr.comm.overlap_log
                out["log"] = log
                out["split_n"] = (tr.comm.n1, tr.comm.n2)
                if trace_path and rank == 0:
                    import json
                    ev = []
                    t0 = log[0]["b1_issue"]
                    for i, r in enumerate(log[1:], 1):
                        us = lambda t: (t - t0) * 1e6
                        ev.append(dict(name=f"bucket-1 all-reduce (u{i}, {r['n1']} grads + fitness + counters)",
                                       ph="X", pid=rank, tid="comm (gloo)", ts=us(r["b1_issue"]),
                                       dur=us(r["b1_done"]) - us(r["b1_issue"])))
                        ev.append(dict(name=f"first-layer backward graph (u{i}, {r['tail_gpu_ms']:.3f} ms on the GPU)",
                                       ph="X", pid=rank, tid="compute stream", ts=us(r["tail_enqueue"]),
                                       dur=r["tail_gpu_ms"] * 1e3))
                        ev.append(dict(name=f"bucket-2 all-reduce + unpack (u{i}, {r['n2']} grads)", ph="X", pid=rank,
                                       tid="comm (gloo)", ts=us(r["b1_done"]),
                                       dur=max(0.0, us(r["b_all_done"]) - us(r["b1_done"]))))
                    with open(trace_path, "w") as f:
                        json.dump({"traceEvents": ev}, f)
        q.put((rank, out))
        ctx.destroy()
    except Exception:   # pragma: no cover
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))


def _run_ranks(world, updates, trace_path=None, dtype="fp32", preset_name="pong", density=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_overlap_worker, args=(r, world, port, q, updates, trace_path, dtype, preset_name, density))
          for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(60)
    for r in range(world):
        assert "error" not in res[r], res[r].get("error")
    return res


def test_overlapped_allreduce_is_bit_equal_to_serial(hip_lib):
    """Two gloo ranks: the split exchange (bucket 1 reduced while the first layer's weight gradient runs) gives
    bit-identical weights, RMSProp slots and GA state to the single-bucket exchange; bucket 1 is still in flight
    when the first-layer backward is enqueued (the overlap)."""
    res = _run_ranks(2, 10, os.environ.get("PATHNET_OVERLAP_TRACE"))
    for r in range(2):
        o, s = res[r]["overlap"], res[r]["serial"]
        assert np.array_equal(o["flat"], s["flat"]) and np.array_equal(o["ms"], s["ms"])
        assert o["gen"] == s["gen"] and np.array_equal(o["geno"], s["geno"])
        n1, n2 = res[r]["split_n"]
        assert n1 > 0 and n2 > 0
        log = res[r]["log"]
        assert len(log) == 10
        assert all(x["b1_issue"] <= x["tail_enqueue"] <= x["b_all_done"] for x in log)
        assert sum(x["tail_enqueue"] < x["b1_done"] for x in log) >= 5      # tail issued before bucket 1 finished
    assert np.array_equal(res[0]["overlap"]["flat"], res[1]["overlap"]["flat"])


def test_overlapped_allreduce_fp32x_matches_serial_and_replicas_agree(hip_lib):
    """The bench engine (fp32x, frame ring) on 2 ranks: the overlapped split exchange vs the single bucket within the
    fp32x budget (float atomics: not bitwise run to run), and within each mode the two replicas bit-identical (every
    rank applies the same all-reduced gradient)."""
    res = _run_ranks(2, 8, dtype="fp32x")
    for r in range(2):
        o, s = res[r]["overlap"], res[r]["serial"]
        d = np.linalg.norm(o["flat"] - s["flat"]) / np.linalg.norm(s["flat"])
        assert d < 1e-5, d
        assert res[r]["split_n"][0] > 0 and res[r]["split_n"][1] > 0
    for mode in ("overlap", "serial"):
        assert np.array_equal(res[0][mode]["flat"], res[1][mode]["flat"]), mode
        assert np.array_equal(res[0][mode]["geno"], res[1][mode]["geno"]), mode


def test_static_and_exact_exchange_plans_agree_bitwise(hip_lib):
    """The two all-reduce plans of the pipelined exchange (trainer._plan_exchange): every trainable module (static,
    no device read-back) vs the exact module union read back from the device GA.  fp32 (fixed-order reductions):
    the same weights, RMSProp slots and genotypes bit for bit, with tournaments firing."""
    st = _run_ranks(2, 8, density=0.0)
    ex = _run_ranks(2, 8, density=2.0)
    for r in range(2):
        assert st[r]["overlap"]["plan_mode"] == "static" and ex[r]["overlap"]["plan_mode"] == "exact"
        for mode in ("overlap", "serial"):
            assert np.array_equal(st[r][mode]["flat"], ex[r][mode]["flat"]), mode
            assert np.array_equal(st[r][mode]["ms"], ex[r][mode]["ms"]), mode
            assert np.array_equal(st[r][mode]["geno"], ex[r][mode]["geno"]), mode
        assert st[r]["overlap"]["gen"] > 0


def test_reference_lstm_preset_overlapped_exchange_two_ranks(hip_lib):
    """The reference network (L=4 trunk + fused fp32x LSTM, synthetic Alien on the frame ring) on 2 gloo ranks with
    the overlapped split exchange (bucket 1 = layers >= 1 + LSTM + heads + fitness + counters, reduced while the first
    layer's weight gradient runs): within the fp32x budget of the single-bucket exchange, replicas bit-identical."""
    res = _run_ranks(2, 6, dtype="fp32x", preset_name="reference")
    for r in range(2):
        o, s = res[r]["overlap"], res[r]["serial"]
        assert o["lstm"], "the reference preset must run the fused HIP LSTM"
        d = np.linalg.norm(o["flat"] - s["flat"]) / np.linalg.norm(s["flat"])
        assert d < 1e-5, d
        assert res[r]["split_n"][0] > 0 and res[r]["split_n"][1] > 0
    for mode in ("overlap", "serial"):
        assert np.array_equal(res[0][mode]["flat"], res[1][mode]["flat"]), mode


def _strong_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), PATHNET_DIST_BACKEND="gloo")
    torch.set_num_threads(2)
    try:
        from pathnet_gym_amd.parallel.dist import init_distributed
        ctx = init_distributed()
        q.put((rank, _strong_run(ctx)))
        ctx.destroy()
    except Exception:   # pragma: no cover
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))


def _strong_run(ctx, updates=8):
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    from pathnet_gym_amd.config import preset
    cfg = preset("pong")
    cfg.paths_total, cfg.envs_per_path, cfg.a2c.t_max = 8, 16, 4
    cfg.ga.backend = "device"
    cfg.ga.concurrent_tournaments = 2
    cfg.ga.fitness_window = 2
    cfg.net.N = 2
    cfg.compute_dtype = "fp32"
    tr = PathNetTrainer(cfg, device=ctx.device, ctx=ctx)
    tr.env.max_episode_steps = 6
    hist = []
    for _ in range(updates):
        st = tr.update()
        hist.append((st.episodes, st.tournaments))
    tr.flush()
    torch.cuda.synchronize()
    return {"flat": tr.model.store.flat.detach().cpu().numpy().copy(), "geno": tr.pop.genotypes.copy(),
            "gen": tr.pop.generation, "step": tr.global_step, "P": tr.P, "hist": hist}


def test_strong_scaling_two_ranks_reproduce_one_gpu_hip_engine(hip_lib):
    """Strong scaling on the HIP engine (fp32, device GA, pipelined, overlapped exchange): 2 gloo ranks x 4 paths
    (paths_total = 8) against one process with the 8 paths: same env streams and sampled actions (keyed by the global
    env index), the same GA decisions; weights equal up to the gradient's summation order."""
    from pathnet_gym_amd.parallel.dist import DistContext
    one = _strong_run(DistContext(device=torch.device("cuda", 0)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_strong_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(60)
    for r in range(2):
        assert "error" not in res[r], res[r].get("error")
        assert res[r]["P"] == 4
    two = res[0]
    assert one["P"] == 8 and one["gen"] > 0
    assert two["gen"] == one["gen"] and two["step"] == one["step"] and two["hist"] == one["hist"]
    assert np.array_equal(two["geno"], one["geno"])
    d = np.linalg.norm(two["flat"] - one["flat"]) / np.linalg.norm(one["flat"])
    assert d < 1e-5, d
    assert np.array_equal(res[0]["flat"], res[1]["flat"])


def test_four_gloo_ranks_tournaments_fire_and_replicas_agree(hip_lib):
    res = _run_ranks(4, 12)
    gens = [res[r]["overlap"]["gen"] for r in range(4)]
    assert gens[0] > 0 and len(set(gens)) == 1, gens
    for r in range(1, 4):
        assert np.array_equal(res[0]["overlap"]["flat"], res[r]["overlap"]["flat"])
        assert np.array_equal(res[0]["overlap"]["geno"], res[r]["overlap"]["geno"])


def _resume_worker(rank, world, port, q, path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), PATHNET_DIST_BACKEND="gloo")
    torch.set_num_threads(2)
    try:
        from pathnet_gym_amd.algo.trainer import PathNetTrainer
        from pathnet_gym_amd.config import preset
        from pathnet_gym_amd.parallel.dist import init_distributed
        from pathnet_gym_amd.utils import checkpoint as ckpt
        ctx = init_distributed()

        def make():
            cfg = preset("pong")
            cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 4, 16, 4
            cfg.ga.backend = "device"
            cfg.ga.concurrent_tournaments = 2
            cfg.ga.fitness_window = 2
            cfg.net.N = 2
            cfg.compute_dtype = "fp32"
            tr = PathNetTrainer(cfg, device=ctx.device, ctx=ctx)
            tr.env.max_episode_steps = 6
            return tr
        a = make()
        for _ in range(6):
            a.update()
        a.flush()
        ckpt.save(a, path)
        ctx.barrier()
        for _ in range(6):
            a.update()
        a.flush()
        torch.cuda.synchronize()
        out = {"flat_a": a.model.store.flat.detach().cpu().numpy().copy(), "gen_a": a.pop.generation,
               "geno_a": a.pop.genotypes.copy()}
        del a
        b = make()
        ckpt.load(b, path)
        for _ in range(6):
            b.update()
        b.flush()
        torch.cuda.synchronize()
        out.update(flat_b=b.model.store.flat.detach().cpu().numpy().copy(), gen_b=b.pop.generation,
                   geno_b=b.pop.genotypes.copy())
        q.put((rank, out))
        ctx.destroy()
    except Exception:   # pragma: no cover
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))


def test_two_gloo_ranks_checkpoint_resume_is_exact(hip_lib, tmp_path):
    """Multi-rank checkpoint -> resume (rank-0 global state + one file per rank: env, engine counters, fitness
    windows): 6 updates, save, 6 more == a fresh trainer that loads the checkpoint and runs the same 6 (fp32 engine,
    device GA with tournaments firing, pipelined, overlapped all-reduce)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    path = str(tmp_path / "ck.safetensors")
    ps = [ctx.Process(target=_resume_worker, args=(r, 2, port, q, path)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(60)
    for r in range(2):
        o = res[r]
        assert "error" not in o, o.get("error")
        assert o["gen_a"] > 0 and o["gen_a"] == o["gen_b"]
        assert np.array_equal(o["geno_a"], o["geno_b"])
        assert np.array_equal(o["flat_a"], o["flat_b"])
