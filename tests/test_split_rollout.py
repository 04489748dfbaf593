"""Split rollout (TrainConfig.rollout_groups, runtime/engine.py ``_rollout_split``) on an MI355X.

The population is stepped as path groups on their own HIP streams (branches of the rollout hipGraph).  Every
kernel of a group computes exactly the rows the single-stream rollout computes for those paths (global RNG
keys, per-path tiling), so with fixed-order gradient reductions the whole training run must be bit-identical
to the one-stream run: observations, sampled actions, logits, weights and gradients.
"""
import pytest
import torch

from pathnet_gym_amd.config import preset

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(groups, mode, updates=4):
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    cfg = preset("pong")
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 8, 16, 5
    cfg.ga.concurrent_tournaments = 1
    cfg.ga.backend = "device"
    cfg.compute_dtype = "fp32" if mode == "fp32" else "bf16"
    cfg.deterministic = mode != "fp32"
    cfg.rollout_groups = groups
    tr = PathNetTrainer(cfg, device=DEV)
    assert tr.engine.groups == groups
    tr.env.max_episode_steps = 7          # episode ends + auto-resets inside the compared rollouts
    for _ in range(updates):              # eager, capture, replays
        tr.update()
    tr.flush()
    torch.cuda.synchronize()
    e = tr.engine
    assert e.g_rollout is not None
    return {"w": tr.model.store.flat.detach().clone(), "g": e.grad_flat.clone(), "obs": e.obs_stacks().clone(),
            "actions": e.actions.clone(), "logits": e.logits.clone(), "values": e.values.clone(),
            "rewards": e.rewards.clone(), "dones": e.dones.clone(), "fitness": e.fitness.clone()}


@pytest.mark.parametrize("mode", ["bf16_deterministic", "fp32"])
@pytest.mark.parametrize("groups", [2, 4])
def test_split_rollout_is_bit_identical(hip_lib, mode, groups):
    ref = _run(1, mode)
    got = _run(groups, mode)
    for k in ref:
        assert torch.equal(ref[k], got[k]), (k, float((ref[k].float() - got[k].float()).abs().max()))


def test_split_rollout_default_mode_rollout_matches(hip_lib):
    """Default (atomic-wgrad) bf16 mode: the FIRST update's rollout does not depend on any gradient, so its
    observations, actions and logits are bit-identical between one and two streams."""
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    out = []
    for groups in (1, 2):
        cfg = preset("pong")
        cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 8, 16, 5
        cfg.rollout_groups = groups
        cfg.use_graph = False
        tr = PathNetTrainer(cfg, device=DEV)
        e = tr.engine
        e.rollout_backward()
        torch.cuda.synchronize()
        out.append((e.obs_stacks().clone(), e.actions.clone(), e.logits.clone(), [a.clone() for a in e.acts],
                    [b.clone() for b in e.bits]))
    (o1, a1, l1, x1, b1), (o2, a2, l2, x2, b2) = out
    assert torch.equal(o1, o2) and torch.equal(a1, a2) and torch.equal(l1, l2)
    for u, v in zip(x1, x2):
        assert torch.equal(u, v)
    for u, v in zip(b1, b2):
        assert torch.equal(u, v)


@pytest.mark.parametrize("graph", [False, True])
def test_obs_double_buffer_carries_the_bootstrap_stack(hip_lib, graph):
    """The last env step of a rollout writes the next rollout's step-0 stacks into the other observation buffer
    (no obs[0] <- obs[T] copy): after every optimizer step, obs_stack(0) is exactly the previous rollout's
    bootstrap input, through the eager update, the capture and replays of both parity graphs."""
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    cfg = preset("pong")
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 4, 16, 3
    cfg.use_graph = graph
    tr = PathNetTrainer(cfg, device=DEV)
    e = tr.engine
    tr.env.max_episode_steps = 4
    pars = []
    for _ in range(5):
        pars.append(e._par)
        e.rollout_backward()
        boot = e.obs_stack(e.T).clone()
        e.optimizer_step(1e-4)
        torch.cuda.synchronize()
        assert torch.equal(e.obs_stack(0), boot)
    assert pars == [0, 1, 0, 1, 0]
    if graph:
        assert len(e.g_rollouts) == 2


def test_rollout_groups_rejects_unsupported():
    """Frame ring / LSTM / torch-stepped games keep one stream; asking for more raises before any launch."""
    if not torch.cuda.is_available():
        pytest.skip("needs the HIP engine")
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    cfg = preset("pong")
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 8, 16, 5
    cfg.frame_ring = True
    cfg.rollout_groups = 0
    tr = PathNetTrainer(cfg, device=DEV)
    assert tr.engine.groups == 1
    cfg.rollout_groups = 2
    with pytest.raises(ValueError):
        PathNetTrainer(cfg, device=DEV)


def _run_x3_ring(groups, graph, updates=4, paths=8):
    """fp32x on the frame ring with a zero learning rate: the weights never move, so every rollout is a pure function
    of the (deterministic) env and GA state and the float-atomic gradient order cannot leak into later updates."""
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    cfg = preset("pong")
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = paths, 16, 5
    cfg.compute_dtype = "fp32x"
    cfg.frame_ring = True
    cfg.use_graph = graph
    cfg.ga.backend = "device"
    cfg.ga.concurrent_tournaments = 2
    cfg.a2c.lr = 0.0
    cfg.rollout_groups = groups
    tr = PathNetTrainer(cfg, device=DEV)
    e = tr.engine
    assert e.ring and e.groups == (groups or e.groups)
    tr.env.max_episode_steps = 7          # episode ends + auto-resets inside the compared rollouts
    snaps = []
    for _ in range(updates):              # eager, capture, replays (the device GA fires tournaments in between)
        tr.update()
        torch.cuda.synchronize()
        # the next rollout's first stack (the env state both must agree on; the ring's later slots hold frames of an
        # earlier rollout, laid out differently by the one-group modular ring and the two-group copied ring)
        snaps.append({"obs": e.obs_stacks(1).clone(), "actions": e.actions.clone(), "logits": e.logits.clone(),
                      "values": e.values.clone(), "rewards": e.rewards.clone(), "dones": e.dones.clone(),
                      "acts": [a.clone() for a in e.acts], "bits": [b.clone() for b in e.bits],
                      "act_idx": tr.model.act_idx.clone()})
    tr.flush()
    return tr, snaps


@pytest.mark.parametrize("graph", [False, True])
def test_x3_ring_split_rollout_is_bit_identical(hip_lib, graph):
    """fp32x frame ring, two path groups (ranged ring env step, ring_fwd / conv23_fwd at the group's base, the
    module-major fc forward on group inverse lists): every update's observations, actions, logits, activations and
    ReLU bits equal the one-stream rollout's, through the eager update, the capture and replays, and across the
    genotype changes of device-GA tournaments."""
    _, ref = _run_x3_ring(1, graph)
    tr, got = _run_x3_ring(2, graph)
    assert tr.engine.groups == 2
    assert not torch.equal(ref[0]["act_idx"], ref[-1]["act_idx"]) or tr.pop.generation > 0
    for u, (a, b) in enumerate(zip(ref, got)):
        for k in a:
            if isinstance(a[k], list):
                for i, (x, y) in enumerate(zip(a[k], b[k])):
                    assert torch.equal(x, y), (u, k, i)
            else:
                assert torch.equal(a[k], b[k]), (u, k)


def test_x3_ring_auto_groups(hip_lib, monkeypatch):
    """rollout_groups = 0 (auto): one group (measured: two never paid, runtime/engine.py _rollout_groups);
    PATHNET_AUTO_GROUP_MAX_PATHS=16 picks two at <= 16 paths on the fp32x frame ring, one at 32."""
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    for limit, paths, want in (("0", 8, 1), ("16", 8, 2), ("16", 16, 2), ("16", 32, 1)):
        monkeypatch.setenv("PATHNET_AUTO_GROUP_MAX_PATHS", limit)
        cfg = preset("pong")
        cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = paths, 16, 2
        cfg.compute_dtype = "fp32x"
        cfg.frame_ring = True
        cfg.rollout_groups = 0
        assert PathNetTrainer(cfg, device=DEV).engine.groups == want, (limit, paths)
