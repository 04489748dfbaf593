"""A2C returns/loss, the analytic loss gradient used by the HIP kernel, TF-RMSProp."""
import math

import numpy as np
import torch

from pathnet_gym_amd.algo.a2c_math import a2c_loss, nstep_returns
from pathnet_gym_amd.algo.optim import RMSPropTF, anneal_lr
from pathnet_gym_amd.config import PathNetConfig, LayerSpec, log_uniform
from pathnet_gym_amd.models.pathnet import ParamLayout


def test_log_uniform_lr0():
    assert abs(log_uniform(1e-4, 1e-2, 0.4226) - 7.0e-4) < 2e-5     # constants.py:24 "around 7e-4"


def test_nstep_returns_hand_example():
    # T=3, one env, gamma=0.5, rewards [1, 5(clipped->1), -2(clipped->-1)], bootstrap 4
    r = torch.tensor([[1.0], [5.0], [-2.0]])
    v = torch.tensor([[0.5], [0.25], [1.0]])
    d = torch.zeros(3, 1, dtype=torch.bool)
    R, adv = nstep_returns(r, v, d, torch.tensor([4.0]), gamma=0.5)
    # R2 = -1 + 0.5*4 = 1 ; R1 = 1 + 0.5*1 = 1.5 ; R0 = 1 + 0.75 = 1.75
    assert torch.allclose(R[:, 0], torch.tensor([1.75, 1.5, 1.0]))
    assert torch.allclose(adv[:, 0], torch.tensor([1.25, 1.25, 0.0]))
    # terminal at t=1 -> no bootstrap across it
    d[1, 0] = True
    R, _ = nstep_returns(r, v, d, torch.tensor([4.0]), gamma=0.5)
    assert torch.allclose(R[:, 0], torch.tensor([1.5, 1.0, 1.0]))


def test_gae_lambda_one_equals_nstep():
    g = torch.Generator().manual_seed(0)
    r = torch.randn(7, 5, generator=g)
    v = torch.randn(7, 5, generator=g)
    d = torch.rand(7, 5, generator=g) < 0.2
    b = torch.randn(5, generator=g)
    R1, A1 = nstep_returns(r, v, d, b, 0.9, 1.0)
    R2, A2 = nstep_returns(r, v, d, b, 0.9, 0.999999)
    assert torch.allclose(A1, A2, atol=1e-4)


def test_loss_matches_reference_definition():
    logits = torch.tensor([[1.0, 2.0, 0.5]])
    v = torch.tensor([0.3])
    a = torch.tensor([1])
    R = torch.tensor([2.0])
    adv = R - v
    loss, lp, lv, ent = a2c_loss(logits, v, a, R, adv, 0.01, 0.5)
    pi = torch.softmax(logits, -1)
    log_pi = torch.log(pi)
    H = -(pi * log_pi).sum()
    ref_pol = -(log_pi[0, 1] * adv[0] + 0.01 * H)
    ref_val = 0.5 * 0.5 * (R - v) ** 2          # 0.5 * tf.nn.l2_loss == 0.25 * sum sq
    assert torch.allclose(loss, ref_pol + ref_val[0])


def test_analytic_logit_gradient_used_by_hip_kernel():
    """dz_j = w*(-adv*(1[j==a]-pi_j) + beta*pi_j*(log pi_j + H)); dv = w*coef*(v-R) (csrc/heads.hip)."""
    g = torch.Generator().manual_seed(2)
    n, A = 16, 6
    z = torch.randn(n, A, generator=g, requires_grad=True)
    v = torch.randn(n, generator=g, requires_grad=True)
    a = torch.randint(0, A, (n,), generator=g)
    R = torch.randn(n, generator=g)
    adv = R - v.detach()
    w = 0.25
    loss, *_ = a2c_loss(z, v, a, R, adv, 0.01, 0.5, torch.full((n,), w))
    loss.backward()
    pi = torch.softmax(z.detach(), -1)
    lp = torch.log(pi)
    H = -(pi * lp).sum(1, keepdim=True)
    oh = torch.nn.functional.one_hot(a, A).float()
    dz = w * (-adv[:, None] * (oh - pi) + 0.01 * pi * (lp + H))
    dv = w * 0.5 * (v.detach() - R)
    assert torch.allclose(z.grad, dz, atol=1e-6)
    assert torch.allclose(v.grad, dv, atol=1e-6)


def _layout():
    cfg = PathNetConfig(L=2, M=3, N=1, input_shape=(4,), layers=[LayerSpec("fc", 8), LayerSpec("fc", 8)],
                        trunk_scale="none", num_actions=2)
    return ParamLayout(cfg)


def test_rmsprop_tf_semantics_and_per_tensor_clip():
    lay = _layout()
    w = torch.randn(lay.numel)
    opt = RMSPropTF(lay, w.clone(), decay=0.99, momentum=0.0, epsilon=0.1, clip_norm=40.0)
    g = torch.randn(lay.numel) * 50
    w0 = opt.flat.clone()
    opt.step(g, 7e-4)
    for s in lay.segments:
        gs = g[s.offset:s.offset + s.numel]
        n = gs.norm()
        gc = gs * 40.0 / max(float(n), 40.0)                     # tf.clip_by_norm per tensor
        ms = 0.99 * 1.0 + 0.01 * gc * gc                          # rms slot initialised to 1.0
        upd = 7e-4 * gc / torch.sqrt(ms + 0.1)                     # epsilon inside the sqrt
        assert torch.allclose(w0[s.offset:s.offset + s.numel] - opt.flat[s.offset:s.offset + s.numel], upd,
                              atol=1e-6)


def test_rmsprop_frozen_segments_untouched_and_zero_grad_decays_ms():
    lay = _layout()
    w = torch.randn(lay.numel)
    opt = RMSPropTF(lay, w.clone())
    frozen = np.zeros((2, 3), np.float32)
    frozen[0, 1] = 1
    opt.set_frozen(frozen)
    g = torch.zeros(lay.numel)
    s_fro = lay.by_name["layer0.module1.weight"]
    s_live = lay.by_name["layer0.module0.weight"]
    g[s_fro.offset:s_fro.offset + s_fro.numel] = 1.0
    before = opt.flat.clone()
    opt.step(g, 1e-2)
    assert torch.equal(opt.flat[s_fro.offset:s_fro.offset + s_fro.numel], before[s_fro.offset:s_fro.offset + s_fro.numel])
    assert torch.allclose(opt.ms[s_live.offset:s_live.offset + s_live.numel], torch.full((s_live.numel,), 0.99))
    assert torch.equal(opt.ms[s_fro.offset:s_fro.offset + s_fro.numel], torch.ones(s_fro.numel))


def test_anneal_modes():
    assert anneal_lr(1.0, 50, 100, 0, "global") == 0.5
    assert anneal_lr(1.0, 150, 100, 100, "global") == 0.0        # reference quirk: lr=0 in task 2
    assert anneal_lr(1.0, 150, 100, 100, "per_task") == 0.5
    assert anneal_lr(1.0, 150, 100, 100, "none") == 1.0
