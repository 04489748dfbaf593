"""Pipelined device-GA mode on the GPU: host runs ahead of two hipGraph replays per update.

Regression for the captured-memset race recorded in profiles/r2_graph_memset_race.md: the episode counters
written by the rollout graph must stay plausible for thousands of un-synchronised updates.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_pipelined_device_ga_counters_stay_sane(hip_lib):
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    from pathnet_gym_amd.config import preset
    cfg = preset("pong")
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 16, 16, 5
    cfg.ga.backend = "device"
    cfg.ga.concurrent_tournaments = 1
    tr = PathNetTrainer(cfg, device="cuda")
    assert tr.pipelined and tr.engine.use_graph
    comm = tr.comm
    P = comm.P_total
    n = 6000
    hist = torch.zeros(n + 1, P + 4, device="cuda")
    orig = comm.exchange_async
    k = [0]

    def ex(*a, **kw):
        h = orig(*a, **kw)
        hist[k[0]].copy_(comm.small_dev)
        k[0] += 1
        return h
    comm.exchange_async = ex
    eps = 0
    for _ in range(n):
        st = tr.update()
        eps += st.episodes
        assert np.isnan(st.mean_return) or abs(st.mean_return) <= 21.0, st
    tr.flush()
    torch.cuda.synchronize()
    H = hist[:k[0]].cpu().numpy()
    cnt, ret = H[:, P + 1], H[:, P + 2]
    assert eps > 0 and cnt.sum() > 0
    assert (np.abs(ret) <= 21.0 * np.maximum(cnt, 1.0)).all(), np.nonzero(np.abs(ret) > 21.0 * np.maximum(cnt, 1.0))[0][:5]
    fit = H[:, :P]
    assert ((fit == -1000.0) | (np.abs(fit) <= 21.0)).all()


def test_frozen_modules_bit_identical_across_task2_updates_hip(hip_lib):
    """Continual learning on the HIP engine: after task 1 freezes its winner path (and per-task head),
    task-2 updates (device GA, pipelined, hipGraphs) leave every frozen parameter bit-identical and
    keep the frozen modules expressed in every task-2 path (doom_pathnet.py:274-293)."""
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    from pathnet_gym_amd.config import preset
    cfg = preset("atari4")
    cfg.tasks = ["Pong", "Pong"]
    cfg.net.num_tasks = 2
    cfg.net.per_task_heads = True
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 8, 16, 4
    cfg.ga.backend = "device"
    cfg.ga.concurrent_tournaments = 2
    tr = PathNetTrainer(cfg, device="cuda")
    for _ in range(30):
        tr.update()
    winner, frozen = tr.end_task()
    tr._start_task(1)
    lay = tr.model.store.layout
    keep = torch.zeros(lay.numel, dtype=torch.bool)
    for s in lay.segments:
        if (s.layer >= 0 and frozen[s.layer, s.module] > 0.5) or s.task == 0:
            keep[s.offset:s.offset + s.numel] = True
    keep = keep.cuda()
    before = tr.model.store.flat.detach()[keep].clone()
    other0 = tr.model.store.flat.detach()[~keep].clone()
    for _ in range(40):
        tr.update()
    tr.flush()
    torch.cuda.synchronize()
    after = tr.model.store.flat.detach()
    assert torch.equal(after[keep], before)
    assert not torch.equal(after[~keep], other0)                 # task 2 does train the rest
    geno = tr.engine.ga_dev["geno"].cpu().numpy() | tr.engine.ga_dev["frozen"].cpu().numpy()[None]
    assert (geno[:, frozen > 0.5] == 1).all()
    assert (tr.model.mask.cpu().numpy()[:, frozen > 0.5] == 1).all()


@pytest.mark.gpu
def test_light_checkpoint_resume_restacks_current_frame(hip_lib, tmp_path):
    """Continuation checkpoints (scripts/solve.py): no frame stacks, no momentum slots (momentum 0); the resumed trainer has
    the same weights, RMSProp slots, GA state and counters, and every env's stack is its current frame x 4."""
    import numpy as np
    import torch
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    from pathnet_gym_amd.config import preset
    from pathnet_gym_amd.utils import checkpoint as ckpt

    def make():
        cfg = preset("pong")
        cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 4, 16, 4
        cfg.ga.backend = "device"
        cfg.compute_dtype = "fp32x"
        cfg.frame_ring = True
        return PathNetTrainer(cfg, device="cuda")
    a = make()
    for _ in range(3):
        a.update()
    a.flush()
    p = str(tmp_path / "ck.safetensors")
    ckpt.save(a, p, light=True)
    from safetensors import safe_open
    with safe_open(p + ".rank0.safetensors", framework="pt") as f:
        assert "engine.obs0" not in f.keys()
    with safe_open(p, framework="pt") as f:
        assert not any(k.endswith("/RMSProp_1") for k in f.keys())
    b = make()
    ckpt.load(b, p)
    assert torch.equal(a.model.store.flat, b.model.store.flat) and torch.equal(a.opt.ms, b.opt.ms)
    assert np.array_equal(a.pop.genotypes, b.pop.genotypes) and a.updates == b.updates
    st = b.engine.obs_stack(0).view(b.P * b.E, -1, 4)
    assert torch.equal(st[..., 0], st[..., 3]) and st.float().mean() > 0
    b.update()
    b.flush()
    assert torch.isfinite(b.model.store.flat).all()


@pytest.mark.gpu
def test_light_checkpoint_of_a_hip_game_on_the_frame_ring(hip_lib, tmp_path):
    """The same continuation checkpoint with a HIP synthetic game (csrc/games.hip) on the frame ring: the game's
    kernel-side state is synced through its own unpacker (not Pong's), and the resumed trainer steps on."""
    import torch
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    from pathnet_gym_amd.config import preset
    from pathnet_gym_amd.utils import checkpoint as ckpt

    def make():
        cfg = preset("atari4")
        cfg.tasks = ["Breakout"]
        cfg.env = "Breakout"
        cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 4, 16, 4
        cfg.ga.backend = "device"
        cfg.compute_dtype = "fp32x"
        cfg.frame_ring = True
        return PathNetTrainer(cfg, device="cuda")
    a = make()
    assert a.engine.ring and a.env.supports_ring
    for _ in range(3):
        a.update()
    a.flush()
    p = str(tmp_path / "ck.safetensors")
    ckpt.save(a, p, light=True)
    b = make()
    ckpt.load(b, p)
    assert torch.equal(a.model.store.flat, b.model.store.flat)
    st = b.engine.obs_stack(0).view(b.P * b.E, -1, 4)
    assert torch.equal(st[..., 0], st[..., 3]) and st.float().mean() > 0
    b.update()
    b.flush()
    assert torch.isfinite(b.model.store.flat).all()
