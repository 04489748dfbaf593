"""The multi-rank code paths on a ONE-rank process group (DistContext.forced, init_distributed(force=True)).

A world-size-1 process group runs every collective the 8-GPU job uses -- the packed active-module all-reduce, the
overlapped two-bucket exchange (exchange_async_split), all_gather_into_tensor, the RCCL barrier with device_ids,
the max-over-ranks timer -- on one device.  Reducing over one rank is the identity, so a trainer on the forced group
must reproduce the trainer without a group: bit for bit on the deterministic engines, to the fp32x budget on fp32x
(its weight gradients use float atomics).  The GPU test runs this over RCCL ("nccl"), the CPU test over gloo.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(backend, dtype):
    from pathnet_gym_amd.config import preset
    if backend == "torch":
        cfg = preset("cartpole-cpu")
        cfg.paths, cfg.envs_per_path = 4, 4
        cfg.ga.concurrent_tournaments = 2
        return cfg
    cfg = preset("pong")
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 4, 16, 4
    cfg.backend = "hip"
    cfg.compute_dtype = dtype
    cfg.frame_ring = dtype == "fp32x"
    cfg.ga.backend = "device"
    cfg.ga.concurrent_tournaments = 1
    return cfg


def _run(ctx, backend, dtype, updates=5):
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    tr = PathNetTrainer(_cfg(backend, dtype), ctx=ctx)
    if backend == "hip":
        tr.env.max_episode_steps = 6
    for _ in range(updates):
        tr.update()
    tr.flush()
    split = bool(getattr(tr.engine, "split", False))
    return {"flat": tr.model.store.flat.detach().cpu().numpy().copy(), "geno": tr.pop.genotypes.copy(),
            "gen": tr.pop.generation, "step": tr.global_step, "split": split}


def _worker(q, port, backend, dtypes):
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        torch.set_num_threads(1)
        from pathnet_gym_amd.parallel.dist import init_distributed
        if backend == "hip":
            from pathnet_gym_amd import _build
            _build.build()
        ctx = init_distributed(device="cuda" if backend == "hip" else "cpu", force=True)
        out = {"backend": ctx.backend, "enabled": ctx.enabled, "world": ctx.world}
        x = torch.arange(6.0, device=ctx.device).view(3, 2)
        out["gather_ok"] = bool(torch.equal(ctx.all_gather(x).cpu(), x.cpu()))     # all_gather_into_tensor on RCCL
        ctx.barrier()                                                                  # barrier(device_ids=[..])
        out["max"] = ctx.max_scalar(3.5)
        for dt in dtypes:
            out[dt] = _run(ctx, backend, dt)
        ctx.destroy()
        q.put(out)
    except Exception:   # pragma: no cover
        import traceback
        q.put({"error": traceback.format_exc()})


def _forced(backend, dtypes):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(q, _free_port(), backend, dtypes))
    p.start()
    out = q.get(timeout=400)
    p.join(60)
    assert "error" not in out, out.get("error")
    assert out["enabled"] and out["world"] == 1 and out["gather_ok"] and out["max"] == 3.5
    return out


def test_forced_one_rank_gloo_group_reproduces_no_group():
    from pathnet_gym_amd.parallel.dist import DistContext
    torch.set_num_threads(1)
    out = _forced("torch", ["fp32"])
    assert out["backend"] == "gloo"
    ref = _run(DistContext(), "torch", "fp32")
    a = out["fp32"]
    assert a["gen"] == ref["gen"] and a["step"] == ref["step"]
    assert np.array_equal(a["geno"], ref["geno"])
    assert np.array_equal(a["flat"], ref["flat"])


@pytest.mark.gpu
def test_forced_one_rank_rccl_group_reproduces_no_group(hip_lib):
    """RCCL ("nccl") process group of one rank on cuda:0: the fp32 engine (deterministic) bit-equal to the run without
    a group, fp32x (overlapped split exchange, frame ring, float atomics) within its per-layer budget."""
    from pathnet_gym_amd.parallel.dist import DistContext
    out = _forced("hip", ["fp32", "fp32x"])
    assert out["backend"] == "nccl"
    ctx0 = DistContext(device=torch.device("cuda", 0))
    for dt in ("fp32", "fp32x"):
        ref = _run(ctx0, "hip", dt)
        a = out[dt]
        assert a["split"] and not ref["split"], dt           # the forced run took the overlapped two-bucket path
        assert a["gen"] == ref["gen"] and a["step"] == ref["step"], dt
        assert np.array_equal(a["geno"], ref["geno"]), dt
        if dt == "fp32":
            assert np.array_equal(a["flat"], ref["flat"])
        else:
            d = np.linalg.norm(a["flat"] - ref["flat"]) / np.linalg.norm(ref["flat"])
            assert d < 1e-5, d


@pytest.mark.gpu
def test_forced_rccl_bench_builds_several_trainers(hip_lib, tmp_path):
    """bench.py on a forced one-rank RCCL group: the headline trainer's all-reduces, then a per-rank-shape trainer and
    an in-run-solve trainer that capture their hipGraphs while the process group's watchdog thread still polls the
    earlier collectives' events.  With the default global capture mode such a poll aborted the process
    (hipErrorStreamCaptureUnsupported); the engine captures in thread-local mode (runtime/engine.py CAPTURE_MODE)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PATHNET_DIST_FORCE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--paths", "16", "--paths-total", "16", "--envs", "16",
           "--tmax", "5", "--steps", "3", "--warmup", "2", "--windows", "2", "--per-rank-shapes", "2",
           "--solve-seconds", "8", "--compare-bf16", "0", "--no-verify-build"]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["n_gpus"] == 1 and d["strong_scaling"]["per_rank"]["by_n_gpus"]["2"]["paths_per_gpu"] == 8
    assert d["generations_to_solve_in_run"]["updates_run"] > 0


def test_engine_captures_graphs_thread_local():
    """CPU guard for the capture mode the RCCL watchdog needs (see the GPU test above)."""
    from pathnet_gym_amd.runtime import engine
    assert engine.CAPTURE_MODE == "thread_local"
    src = open(engine.__file__).read()
    assert src.count("capture_error_mode=CAPTURE_MODE") == 3 and src.count("torch.cuda.graph(") == 3
