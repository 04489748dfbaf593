"""Batched external-Gym bridge (envs/gym_bridge.py): semantics vs the reference GameState, trainer learning."""
import numpy as np
import pytest
import torch

from pathnet_gym_amd.envs.game_state import preprocess_numpy
from pathnet_gym_amd.envs.gym_bridge import GymVecEnv, PyCartPole, PyCatch
from pathnet_gym_amd.envs.registry import make


class GymnasiumCartPole(PyCartPole):
    """The same env against the gymnasium API (reset -> (obs, info), 5-tuple step, reset(seed=))."""

    def reset(self, seed=None):
        if seed is not None:
            self.np_random = np.random.RandomState(seed)
        return super().reset(), {}

    def step(self, a):
        o, r, d, info = super().step(a)
        trunc = self.steps >= self.max_episode_steps
        return o, r, d and not trunc, trunc, info

    seed = None          # no classic seed()


def test_real_ale_ids_need_gym_and_say_so():
    with pytest.raises(KeyError, match="gym"):
        make("PongNoFrameskip-v4", num_envs=2)
    with pytest.raises(KeyError, match="gym"):
        make("Alien-v0", num_envs=1)


def test_vector_bridge_matches_host_envs_and_autoresets():
    N = 5
    env = make("PyCartPole-v1", num_envs=N, seed=7)
    assert isinstance(env, GymVecEnv) and env.num_actions == 2 and not env.pixels
    ref = [PyCartPole() for _ in range(N)]
    for i, e in enumerate(ref):
        e.seed(7 + i)
    ref_obs = np.stack([e.reset() for e in ref])
    assert np.allclose(env.state.numpy(), ref_obs)
    rets = np.zeros(N)
    seen = 0
    rng = np.random.RandomState(0)
    for t in range(120):
        a = rng.randint(0, 3, size=N)                    # 2 is out of range -> remapped to 0 (game_state.py:38-39)
        obs, r, d, info = env.step(torch.from_numpy(a))
        for i, e in enumerate(ref):
            o, rr, dd, _ = e.step(int(a[i]) if a[i] < 2 else 0)
            rets[i] += rr
            assert bool(d[i]) == dd
            if dd:
                assert float(info["episode_return"][i]) == rets[i]
                rets[i] = 0
                seen += 1
                o = e.reset()
            else:
                assert float(info["episode_return"][i]) == 0.0
            assert np.allclose(obs[i].numpy(), o, atol=1e-6)
    assert seen > 0


def test_gymnasium_api_is_accepted():
    env = GymVecEnv([GymnasiumCartPole() for _ in range(3)], seed=1)
    for _ in range(40):
        obs, r, d, info = env.step(torch.ones(3, dtype=torch.long))
    assert obs.shape == (3, 4) and torch.isfinite(obs).all()


def test_pixel_bridge_matches_reference_preprocessing():
    """Frames: gray + INTER_LINEAR 160x120 + 4-stack newest last, fresh stack after a reset (game_state.py:41-78)."""
    N = 3
    env = GymVecEnv([PyCatch(balls=2, speed=40) for _ in range(N)], seed=3, no_op_max=0)
    assert env.pixels and env.obs_shape == (160, 120, 4)
    ref = [PyCatch(balls=2, speed=40) for _ in range(N)]
    stacks = []
    for i, e in enumerate(ref):
        e.seed(3 + i)
        x = preprocess_numpy(e.reset())
        stacks.append(np.stack([x] * 4, 2))
    got = env.obs.numpy().astype(np.float32) / 255.0
    assert np.allclose(got, np.stack(stacks), atol=1e-6)
    for t in range(12):
        a = torch.tensor([t % 3, (t + 1) % 3, 2])
        obs, r, d, info = env.step(a)
        for i, e in enumerate(ref):
            f, rr, dd, _ = e.step(int(a[i]))
            if dd:
                x = preprocess_numpy(e.reset())
                stacks[i] = np.stack([x] * 4, 2)
            else:
                stacks[i] = np.concatenate([stacks[i][:, :, 1:], preprocess_numpy(f)[:, :, None]], 2)
            assert float(r[i]) == rr and bool(d[i]) == dd
        assert np.allclose(obs.numpy().astype(np.float32) / 255.0, np.stack(stacks), atol=1e-6)


def test_sharded_bridge_reproduces_the_unsharded_envs():
    """Two ranks owning envs [0, 2) and [2, 4) (set_id_base, as the trainer does with rank * P * E) see exactly the
    seeds, no-op starts and trajectories of one 4-env bridge, and the two ranks' envs differ from each other."""
    def catch_env(n, base):
        e = GymVecEnv([PyCatch(balls=3, speed=30) for _ in range(n)], seed=11, no_op_max=4)
        e.set_id_base(base)
        return e, e.reset().clone()
    whole, o_whole = catch_env(4, 0)
    r0, o0 = catch_env(2, 0)
    r1, o1 = catch_env(2, 2)
    assert torch.equal(torch.cat([o0, o1]), o_whole)
    assert not torch.equal(o0, o1)
    for t in range(15):
        a = torch.tensor([t % 3, 1, 2, (t + 2) % 3])
        ow, rw, dw, iw = whole.step(a)
        oa, ra, da, ia = r0.step(a[:2])
        ob, rb, db, ib = r1.step(a[2:])
        assert torch.equal(torch.cat([oa, ob]), ow) and torch.equal(torch.cat([da, db]), dw)
        assert torch.equal(torch.cat([ia["episode_return"], ib["episode_return"]]), iw["episode_return"])
    # vector obs: rank 1's first env is seeded as global env 2
    v = GymVecEnv([PyCartPole() for _ in range(2)], seed=7)
    v.set_id_base(2)
    ref = PyCartPole()
    ref.seed(7 + 2)
    assert np.allclose(v.reset()[0].numpy(), ref.reset())


def test_trainer_learns_cartpole_through_the_bridge():
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    from pathnet_gym_amd.config import preset
    torch.manual_seed(0)
    cfg = preset("cartpole-cpu")
    cfg.env = "PyCartPole-v1"
    cfg.tasks = ["PyCartPole-v1"]
    cfg.paths, cfg.envs_per_path = 8, 8
    tr = PathNetTrainer(cfg)
    assert isinstance(tr.env, GymVecEnv)
    rets = []
    for _ in range(250):
        st = tr.update()
        if not np.isnan(st.mean_return):
            rets.append(st.mean_return)
    assert np.mean(rets[-20:]) > np.mean(rets[:20]) + 10
    assert tr.pop.generation > 10


# ---------------------------------------------------------------------------
# MI355X: HIP preprocessing kernel behind the bridge, HIP engine driven by host gym envs
# ---------------------------------------------------------------------------
@pytest.mark.gpu
def test_pixel_bridge_hip_push_is_bit_exact(hip_lib):
    N = 4
    cpu = GymVecEnv([PyCatch(balls=2, speed=40) for _ in range(N)], seed=5, no_op_max=3)
    gpu = GymVecEnv([PyCatch(balls=2, speed=40) for _ in range(N)], device="cuda", backend="hip", seed=5,
                    no_op_max=3)
    assert torch.equal(cpu.obs, gpu.obs.cpu())
    for t in range(20):
        a = torch.tensor([(t * 7 + i) % 4 for i in range(N)])
        o1, r1, d1, i1 = cpu.step(a)
        o2, r2, d2, i2 = gpu.step(a.cuda())
        assert torch.equal(o1, o2.cpu()), t
        assert torch.equal(r1, r2.cpu()) and torch.equal(d1, d2.cpu())
        assert torch.equal(i1["episode_return"], i2["episode_return"].cpu())


@pytest.mark.gpu
def test_hip_engine_learns_cartpole_through_the_bridge(hip_lib):
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    from pathnet_gym_amd.config import preset
    cfg = preset("cartpole")
    cfg.env = "PyCartPole-v1"
    cfg.tasks = ["PyCartPole-v1"]
    cfg.paths, cfg.envs_per_path = 8, 16
    cfg.backend = "hip"
    tr = PathNetTrainer(cfg, device="cuda")
    assert isinstance(tr.env, GymVecEnv) and tr.engine is not None and not tr.engine.use_graph
    rets = []
    for _ in range(250):
        st = tr.update()
        if not np.isnan(st.mean_return):
            rets.append(st.mean_return)
    tr.flush()
    assert np.mean(rets[-20:]) > np.mean(rets[:20]) + 10, (np.mean(rets[:20]), np.mean(rets[-20:]))


@pytest.mark.gpu
def test_hip_engine_pixel_update_through_the_bridge(hip_lib):
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    from pathnet_gym_amd.config import preset
    cfg = preset("pong")
    cfg.env = "PyCatch-v0"
    cfg.tasks = ["PyCatch-v0"]
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 4, 16, 4
    cfg.backend = "hip"
    tr = PathNetTrainer(cfg, device="cuda")
    eng = tr.engine
    assert isinstance(tr.env, GymVecEnv) and not eng.use_graph
    for _ in range(3):
        tr.update()
    tr.flush()
    torch.cuda.synchronize()
    assert torch.isfinite(tr.model.store.flat).all()
    # the rollout's newest stack (copied to slot 0 by the optimizer step) is the bridge's current observation
    assert torch.equal(eng.obs_stack(0).view(-1), tr.env.obs.reshape(-1))
    assert float(eng.grad_flat.abs().sum()) > 0
