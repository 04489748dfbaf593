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
