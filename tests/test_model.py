"""Super-network layout + oracle forward semantics (game_ac_network.py)."""
import numpy as np
import torch
import torch.nn.functional as F

from pathnet_gym_amd.config import LayerSpec, PathNetConfig, preset
from pathnet_gym_amd.models.pathnet import (ParamStore, count_params, forward_flops_per_sample, lstm_cell_ref,
                                            trunk_forward_ref)


def test_parameter_counts_match_reference():
    assert count_params(preset("reference").net) == 4_173_955          # LSTM variant
    assert count_params(PathNetConfig(L=4, M=10, N=4)) == 3_648_643     # FF variant
    assert abs(forward_flops_per_sample(PathNetConfig(L=4, M=10, N=4)) / 1e6 - 61.4) < 1.5


def test_layer_shapes_reference_trunk():
    sh = PathNetConfig(L=4, M=10, N=4).layer_shapes()
    assert [s[1] for s in sh] == [(39, 29, 8), (18, 13, 8), (16, 11, 8), (256,)]
    assert sh[3][2] == 1408                                              # last_lin_num


def _explicit_reference(store, x, mask):
    """Per-module loop exactly like game_ac_network.py:378-394 (TF NHWC conv, sum of masked relu)."""
    cfg = store.cfg
    h = x
    for l, spec in enumerate(cfg.layers):
        li = store.layout.layer_info[l]
        outs = []
        for j in range(cfg.M):
            W = store.W(l)[j]
            b = store.b(l)[j]
            if spec.kind == "conv":
                k = spec.kernel
                Wt = W.reshape(k, k, li["cin"], li["cout"]).permute(3, 2, 0, 1)
                y = F.conv2d(h.permute(0, 3, 1, 2), Wt, b, stride=spec.stride).permute(0, 2, 3, 1)
                outs.append(F.relu(y) * mask[:, l, j, None, None, None])
            else:
                y = h.reshape(h.shape[0], -1) @ W + b
                outs.append(F.relu(y) * mask[:, l, j, None])
        h = sum(outs)
    h = h.reshape(h.shape[0], -1)
    return h / cfg.M if cfg.trunk_scale == "M" else h


def test_oracle_matches_explicit_module_loop():
    cfg = PathNetConfig(L=4, M=3, N=2, input_shape=(40, 40, 4),
                        layers=[LayerSpec("conv", 8, 8, 4), LayerSpec("conv", 8, 4, 2), LayerSpec("conv", 8, 1, 1),
                                LayerSpec("fc", 16)])
    st = ParamStore(cfg, "cpu", seed=3)
    x = torch.rand(5, 40, 40, 4)
    mask = torch.randint(0, 2, (5, cfg.L, cfg.M)).float()
    mask[0, 1] = 0                                    # empty layer
    a = trunk_forward_ref(st, x, mask)
    b = _explicit_reference(st, x, mask)
    assert torch.allclose(a, b, atol=1e-5)
    # an empty layer outputs zeros: sample 0's output no longer depends on its input
    x2 = x.clone()
    x2[0] = torch.rand(40, 40, 4)
    assert torch.allclose(trunk_forward_ref(st, x2, mask)[0], a[0])


def test_inactive_modules_get_zero_gradient():
    cfg = PathNetConfig(L=2, M=3, N=1, input_shape=(6,), layers=[LayerSpec("fc", 8), LayerSpec("fc", 8)],
                        trunk_scale="none")
    st = ParamStore(cfg, "cpu", seed=0)
    st.flat.requires_grad_(True)
    mask = torch.zeros(4, 2, 3)
    mask[:, 0, 1] = 1
    mask[:, 1, 2] = 1
    trunk_forward_ref(st, torch.randn(4, 6), mask).sum().backward()
    g = st.flat.grad
    for s in st.layout.segments:
        if s.layer < 0:
            continue
        active = mask[0, s.layer, s.module] > 0
        nz = bool(g[s.offset:s.offset + s.numel].abs().sum() > 0)
        if not active:
            assert not nz, s.name


def test_module2_types_skip_fc_residual():
    cfg = PathNetConfig(L=2, M=3, N=1, input_shape=(8,),
                        layers=[LayerSpec("fc", 8), LayerSpec("fc", 8, module_types=[0, 1, 2])], trunk_scale="none")
    st = ParamStore(cfg, "cpu", seed=1)
    x = torch.randn(3, 8)
    h0 = trunk_forward_ref(st, x, torch.tensor([[[1.0, 0, 0], [0, 0, 0]]]).repeat(3, 1, 1))  # layer1 empty
    assert torch.count_nonzero(h0) == 0
    m_skip = torch.tensor([[[1.0, 0, 0], [1.0, 0, 0]]]).repeat(3, 1, 1)
    m_res = torch.tensor([[[1.0, 0, 0], [0, 0, 1.0]]]).repeat(3, 1, 1)
    h1 = F.relu(x @ st.W(0)[0] + st.b(0)[0])
    assert torch.allclose(trunk_forward_ref(st, x, m_skip), h1, atol=1e-6)      # skip = identity (pathnet.py:141)
    res = F.relu(h1 @ st.W(1)[2] + st.b(1)[2]) + h1                              # residual (pathnet.py:158-166)
    assert torch.allclose(trunk_forward_ref(st, x, m_res), res, atol=1e-6)


def test_lstm_cell_tf_semantics():
    torch.manual_seed(0)
    x, h, c = torch.randn(2, 3), torch.randn(2, 4), torch.randn(2, 4)
    k, b = torch.randn(7, 16), torch.randn(16)
    h2, c2 = lstm_cell_ref(x, h, c, k, b)
    z = torch.cat([x, h], 1) @ k + b
    i, j, f, o = z.split(4, 1)                     # TF BasicLSTMCell order i, j, f, o
    cc = c * torch.sigmoid(f + 1.0) + torch.sigmoid(i) * torch.tanh(j)
    assert torch.allclose(c2, cc) and torch.allclose(h2, torch.tanh(cc) * torch.sigmoid(o))


def test_init_ranges_muupan():
    cfg = PathNetConfig(L=4, M=2, N=1)
    st = ParamStore(cfg, "cpu", seed=0)
    w = st.W(0)
    d = 1 / np.sqrt(256)
    assert float(w.abs().max()) <= d + 1e-6
    pw, pb, vw, vb = st.head()
    assert float(pw.abs().max()) <= 1 / np.sqrt(256) + 1e-6


def test_x3_geometry_support_and_fp32_fallback_reason():
    """fp32x kernels exist for the reference pixel trunk (8,4,3 / 4,2,1 on 160x120x4) and fc widths % 64; any other
    --kernel_num / --stride_size runs the fp32 engine (trainer.precision_note says why) instead of raising."""
    from pathnet_gym_amd.config import PathNetConfig, preset, reference_pixel_layers
    from pathnet_gym_amd.ops.pathnet_ops import x3_unsupported_reason
    assert x3_unsupported_reason(preset("pong").net) is None
    assert x3_unsupported_reason(preset("reference").net) is None
    odd = PathNetConfig(L=4, M=10, N=4, layers=reference_pixel_layers(4, (8, 4, 3), (4, 2, 2)))
    assert "conv layer 2" in x3_unsupported_reason(odd)
    assert "M=12" in x3_unsupported_reason(PathNetConfig(L=4, M=12, N=4))
