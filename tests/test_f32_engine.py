"""fp32 engine mode (csrc/trunk_f32.hip) and the deterministic-reduction switch, on an MI355X.

The reference computes in fp32 (TF default dtype, game_ac_network.py:89-110).  The fp32 mode must therefore
match a PLAIN fp32 PyTorch oracle (no bf16 emulation) to fp32 round-off, and -- like the deterministic bf16
mode -- reproduce an update bit for bit (no fp32 atomics in any gradient reduction).
"""
import numpy as np
import pytest
import torch

from pathnet_gym_amd.algo.a2c_math import a2c_loss, nstep_returns
from pathnet_gym_amd.algo.ga import get_geopath
from pathnet_gym_amd.config import LayerSpec, PathNetConfig, preset
from pathnet_gym_amd.models.acnet import ACPathNet
from pathnet_gym_amd.models.pathnet import ParamStore, heads_ref, trunk_forward_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a = a.float().flatten()
    b = b.float().flatten()
    return float((a - b).norm() / (b.norm() + 1e-12))


def masks_with_edges(P, L, M, N, seed=0):
    rng = np.random.RandomState(seed)
    m = np.stack([get_geopath(L, M, N, rng) for _ in range(P)])
    m[0, 1, :] = 0          # empty layer
    m[1, :, :] = 1          # every module active
    m[2, 0, :] = 0
    m[2, 0, M - 1] = 1      # one (odd) module
    return m


def pixel_cfg():
    return PathNetConfig(L=5, M=10, N=4, input_shape=(160, 120, 4),
                         layers=[LayerSpec("conv", 8, 8, 4), LayerSpec("conv", 8, 4, 2), LayerSpec("conv", 8, 3, 1),
                                 LayerSpec("fc", 256), LayerSpec("fc", 256)],
                         trunk_scale="M", num_actions=6)


def test_f32_trunk_forward_matches_plain_fp32_oracle(hip_lib):
    cfg = pixel_cfg()
    P, E = 4, 16
    m = ACPathNet(cfg, P, DEV, "hip", seed=3, compute_dtype="fp32")
    m.set_paths(masks_with_edges(P, cfg.L, cfg.M, cfg.N))
    assert m.hip.f32 and m.hip.Wc[0].dtype == torch.float32
    g = torch.Generator(device="cpu").manual_seed(0)
    obs = torch.randint(0, 256, (P * E, 160, 120, 4), generator=g, dtype=torch.uint8).to(DEV)
    feat = m.hip.trunk(obs, E)
    with torch.no_grad():
        ref = trunk_forward_ref(m.store, obs.float() / 255.0, m.mask.repeat_interleave(E, 0))
    for p in range(P):
        sl = slice(p * E, (p + 1) * E)
        if ref[sl].norm() == 0:
            assert feat[sl].norm() == 0, p
            continue
        assert rel(feat[sl], ref[sl]) < 2e-5, (p, rel(feat[sl], ref[sl]))


def test_f32_vector_trunk_matches_oracle(hip_lib):
    cfg = preset("cartpole").net
    P, E = 6, 16
    rng = np.random.RandomState(1)
    masks = np.stack([get_geopath(cfg.L, cfg.M, cfg.N, rng) for _ in range(P)])
    m = ACPathNet(cfg, P, DEV, "hip", seed=3, compute_dtype="fp32")
    m.set_paths(masks)
    assert m.hip.geoms[0].ldx == 4          # fp32 vector observations are not padded
    x = torch.randn(P * E, 4, device=DEV)
    feat = m.hip.trunk(x, E)
    with torch.no_grad():
        ref = trunk_forward_ref(m.store, x, m.mask.repeat_interleave(E, 0))
    assert rel(feat, ref) < 2e-5


def _oracle_grad(tr, eng):
    """Autograd of the A2C loss over the engine's stored rollout, plain fp32."""
    cfg = tr.cfg
    T, B = eng.T, eng.B
    a2c = cfg.a2c
    flat = tr.model.store.flat.detach().clone().requires_grad_(True)
    st = ParamStore(cfg.net, DEV, flat=flat)
    x = eng.obs_stacks().reshape((T + 1) * B, 160, 120, 4).float() / 255.0
    mask = tr.model.mask.repeat_interleave(eng.E, 0).repeat(T + 1, 1, 1)
    feat = trunk_forward_ref(st, x, mask)
    logits, values = heads_ref(st, feat)
    assert rel(logits[:T * B], eng.logits[:T].reshape(-1, eng.A)) < 1e-4
    assert rel(values, eng.values[:T + 1].reshape(-1)) < 1e-4
    R, adv = nstep_returns(eng.rewards, eng.values[:T], eng.dones.bool(), eng.values[T], a2c.gamma,
                           a2c.gae_lambda, a2c.reward_clip)
    loss, _, _, _ = a2c_loss(logits[:T * B], values[:T * B], eng.actions[:T].reshape(-1).long(), R.reshape(-1),
                             adv.reshape(-1), a2c.entropy_beta, a2c.value_coef,
                             torch.full((T * B,), eng.weight, device=DEV))
    loss.backward()
    return flat.grad


# measured 0.74e-6 .. 1.09e-6 per layer (profiles/fp32/pytest_f32_v3.log)
F32_LAYER_TOL = 1e-5


def test_f32_engine_gradient_vs_plain_fp32_oracle(hip_lib):
    """Whole-update gradient of the fp32 engine vs fp32 autograd: fp32 round-off per layer, <= 1e-5."""
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    cfg = preset("pong")
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 3, 16, 4
    cfg.use_graph = False
    cfg.compute_dtype = "fp32"
    tr = PathNetTrainer(cfg, device=DEV)
    eng = tr.engine
    assert tr.compute_dtype == "fp32" and eng.acts[0].dtype == torch.float32 and not eng.ring
    tr.env.max_episode_steps = 5
    tr.update()
    eng._rollout_backward_body()
    torch.cuda.synchronize()
    g_ref, g_hip = _oracle_grad(tr, eng), eng.grad_flat
    parts = {}
    for s in tr.model.store.layout.segments:
        key = s.layer if s.layer >= 0 else s.name.split(".")[0]
        parts.setdefault(key, []).append((g_hip[s.offset:s.offset + s.numel], g_ref[s.offset:s.offset + s.numel]))
    layer_err = {k: rel(torch.cat([a for a, _ in v]), torch.cat([b for _, b in v])) for k, v in parts.items()}
    print("fp32 engine vs fp32 oracle, per layer:", {k: f"{v:.2e}" for k, v in layer_err.items()})
    for k, v in layer_err.items():
        assert v < F32_LAYER_TOL, (k, v)
    # negative control: any layer's largest active module gradient x 1.02 breaks the budget
    for l in range(cfg.net.L):
        ws = [s for s in tr.model.store.layout.segments if s.layer == l and s.name.endswith(".weight")]
        s = max(ws, key=lambda x: float(g_ref[x.offset:x.offset + x.numel].norm()))
        bad = g_hip.clone()
        bad[s.offset:s.offset + s.numel] *= 1.02
        segs = [x for x in tr.model.store.layout.segments if x.layer == l]
        e = rel(torch.cat([bad[x.offset:x.offset + x.numel] for x in segs]),
                torch.cat([g_ref[x.offset:x.offset + x.numel] for x in segs]))
        assert e > F32_LAYER_TOL, (l, s.name, e)


@pytest.mark.parametrize("mode", ["fp32", "bf16_deterministic"])
def test_updates_are_bit_reproducible(hip_lib, mode):
    """Two trainers from the same seed produce bit-identical weights after several updates (graph-replayed,
    device GA, pipelined): every gradient reduction runs in a fixed order."""
    from pathnet_gym_amd.algo.trainer import PathNetTrainer

    def run():
        cfg = preset("pong")
        cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 4, 16, 5
        cfg.ga.concurrent_tournaments = 1
        cfg.ga.backend = "device"
        cfg.compute_dtype = "fp32" if mode == "fp32" else "bf16"
        cfg.deterministic = mode != "fp32"
        tr = PathNetTrainer(cfg, device=DEV)
        assert tr.model.hip.deterministic
        tr.env.max_episode_steps = 7
        for _ in range(4):
            tr.update()
        tr.flush()
        torch.cuda.synchronize()
        return tr.model.store.flat.detach().clone(), tr.engine.grad_flat.clone()

    w1, g1 = run()
    w2, g2 = run()
    assert torch.equal(g1, g2), float((g1 - g2).abs().max())
    assert torch.equal(w1, w2), float((w1 - w2).abs().max())


def test_bf16_deterministic_gradient_matches_default_path(hip_lib):
    """The deterministic bf16 weight gradients (ordered fp32 kernels over bf16 activations) agree with the
    default atomic kernels on the same rollout to accumulation round-off."""
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    cfg = preset("pong")
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 3, 16, 4
    cfg.use_graph = False
    cfg.frame_ring = False
    tr = PathNetTrainer(cfg, device=DEV)
    eng = tr.engine
    hp = tr.model.hip
    tr.update()
    eng._rollout_backward_body()
    torch.cuda.synchronize()
    g_default = eng.grad_flat.clone()
    hp.deterministic = True
    # the default engine keeps the conv1 / conv2 output gradients in bf16; the ordered kernels take fp32
    eng.grads = [torch.zeros(g.shape, dtype=torch.float32, device=DEV) for g in eng.grads]
    try:
        eng.grad_flat.zero_()
        L = len(hp.geoms)
        T, B = eng.T, eng.B
        hp.heads_bwd(eng.acts[L - 1][:T].reshape(T * B, -1), eng.dlogits.reshape(T * B, -1),
                     eng.dvalue.reshape(-1), eng.grad_flat, eng.grads[L - 1], task=tr.model.task)
        eng._layer_bwd_all(T)
        torch.cuda.synchronize()
    finally:
        hp.deterministic = False
    for s in tr.model.store.layout.segments:
        a, b = eng.grad_flat[s.offset:s.offset + s.numel], g_default[s.offset:s.offset + s.numel]
        if b.norm() < 1e-7:
            assert a.norm() < 1e-5, s.name
            continue
        # conv1 / fc1: bf16 masked-G (default fc_wgrad_gm) vs fp32 masked-G (ordered kernel) operands
        assert rel(a, b) < 1e-2, (s.name, rel(a, b))
