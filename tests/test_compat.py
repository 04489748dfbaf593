"""Reference-API compatibility layer (pathnet.py, game_ac_network.py, a3c_training_thread.py,
rmsprop_applier.py, input_data.py) -- CPU, plain PyTorch fp32 oracles."""
import gzip
import types

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from pathnet_gym_amd.compat import pathnet as pn
from pathnet_gym_amd.compat.a3c_training_thread import A3CTrainingThread
from pathnet_gym_amd.compat.game_ac_network import GameACPathNetLSTMNetwork, GameACPathNetNetwork
from pathnet_gym_amd.compat.input_data import read_data_sets
from pathnet_gym_amd.compat.rmsprop_applier import RMSPropApplier


def _flags(**kw):
    d = dict(L=4, M=3, N=2, kernel_num="8,4,3", stride_size="4,2,1", task_index=0, use_lstm=False)
    d.update(kw)
    return types.SimpleNamespace(**d)


def test_module_kinds():
    torch.manual_seed(0)
    x = torch.randn(5, 6)
    W, b = torch.randn(6, 6), torch.randn(6)
    assert torch.equal(pn.module2(0, x, [W], [b]), x)                                   # skip
    assert torch.allclose(pn.module2(1, x, [W], [b]), F.relu(x @ W + b))               # fc
    assert torch.allclose(pn.module2(2, x, [W], [b]), F.relu(x @ W + b) + x)           # residual
    assert torch.allclose(pn.nn_layer(x, W, b), x @ W + b)
    img = torch.rand(2, 12, 10, 3)
    Wc, bc = torch.randn(3, 3, 3, 4), torch.randn(4)
    ref = F.relu(F.conv2d(img.permute(0, 3, 1, 2), Wc.permute(3, 2, 0, 1), bc, stride=2)).permute(0, 2, 3, 1)
    assert torch.allclose(pn.conv_module(img, [Wc], [bc], 2), ref, atol=1e-6)


def test_variables_and_backup_roundtrip():
    w = pn.weight_variable([50, 40])
    assert float(w.abs().max()) <= 0.2 + 1e-6
    assert torch.all(pn.bias_variable([7]) == 0.1)
    vs = [w, pn.module_bias_variable([3])[0]]
    bk = pn.parameters_backup(vs)
    with torch.no_grad():
        for v in vs:
            v.add_(1.0)
    pn.parameters_update(None, vs, None, bk)
    assert all(torch.equal(v, b) for v, b in zip(vs, bk))
    s = pn.variable_summaries(w, "w")
    assert set(s) >= {"mean", "stddev", "max", "min", "histogram"}


def test_geopath_helpers_and_ga_ops():
    g = pn.geopath_initializer(3, 5)
    assert torch.all(g == 1)
    np.random.seed(0)
    c = pn.get_geopath(3, 5, 2)
    assert (c.sum(1) == 2).all()
    pn.geopath_insert(None, g, None, c, 3, 5)
    assert np.array_equal(g.numpy(), c)
    m = pn.mutation(c.copy(), 3, 5, 2)
    assert m.shape == (3, 5)
    a, b = pn.select_two_candi(5)
    assert a != b


def test_rmsprop_applier_tf_semantics():
    torch.manual_seed(1)
    v = torch.randn(10)
    v0 = v.clone()
    g = torch.randn(10) * 100            # norm > 40 -> clipped
    opt = RMSPropApplier(learning_rate=0.01, decay=0.99, epsilon=0.1, clip_norm=40.0)
    opt.apply_gradients([v], [g])
    gc = g * 40.0 / g.norm()
    ms = 0.99 * 1.0 + 0.01 * gc * gc           # rms slot initialised to 1.0
    assert torch.allclose(v, v0 - 0.01 * gc / torch.sqrt(ms + 0.1), atol=1e-6)
    assert torch.allclose(opt.get_slot(v, "rms"), ms)


def test_network_vars_and_policy():
    net = GameACPathNetNetwork(0, thread_index=11, FLAGS=_flags())
    L, M = 4, 3
    assert len(net.get_vars()) == 2 * L * M + 4
    fp = np.zeros((L, M))
    fp[0, 1] = fp[3, 2] = 1
    net.set_fixed_path(fp)
    idx = net.get_vars_idx()
    assert len(idx) == 2 * L * M + 4 and sum(idx) == 2 * L * M + 4 - 4
    assert len(net.get_vars()) == sum(idx)
    s = np.random.rand(160, 120, 4).astype(np.float32)
    pi, v = net.run_policy_and_value(None, s)
    assert pi.shape == (18,) and abs(pi.sum() - 1) < 1e-5 and np.isfinite(v)
    pi2, _ = net.run_policy_and_value(s)           # sess-less call style
    assert np.allclose(pi, pi2)
    other = GameACPathNetNetwork(0, thread_index=12, FLAGS=_flags(), seed=5)
    other.sync_from(net)
    assert torch.equal(other.store.flat, net.store.flat)


def test_network_loss_matches_formula():
    net = GameACPathNetNetwork(0, thread_index=13, FLAGS=_flags())
    net.prepare_loss(0.01)
    T = 3
    s = np.random.rand(T, 160, 120, 4).astype(np.float32)
    a = np.eye(18, dtype=np.float32)[[1, 4, 0]]
    td, r = np.array([0.5, -1.0, 2.0], np.float32), np.array([1.0, 0.0, -1.0], np.float32)
    loss = net.loss(s, a, td, r)
    pi, v = net._forward(s)
    lp = torch.log(pi.clamp(1e-20, 1))
    ent = -(pi * lp).sum(1)
    ref = -(((lp * torch.from_numpy(a)).sum(1) * torch.from_numpy(td)) + 0.01 * ent).sum() \
        + 0.25 * ((torch.from_numpy(r) - v) ** 2).sum()
    assert torch.allclose(loss, ref, atol=1e-5)


def test_lstm_network_state_rollback():
    net = GameACPathNetLSTMNetwork(0, thread_index=14, FLAGS=_flags(use_lstm=True))
    s = np.random.rand(160, 120, 4).astype(np.float32)
    h0 = net.lstm_state_out[0].copy()
    net.run_value(s)                                   # rolls back
    assert np.array_equal(net.lstm_state_out[0], h0)
    net.run_policy_and_value(s)                        # advances
    assert not np.array_equal(net.lstm_state_out[0], h0)
    net.reset_state()
    assert not net.lstm_state_out[0].any()
    assert len(net.get_vars()) == 2 * 4 * 3 + 6


def test_a3c_thread_process_trains_unfrozen_only():
    flags = _flags()
    glob = GameACPathNetNetwork(0, thread_index=15, FLAGS=flags)
    opt = RMSPropApplier(learning_rate=7e-4, decay=0.99, epsilon=0.1, clip_norm=40.0)
    th = A3CTrainingThread(0, glob, 0, 7e-4, None, opt, 10 ** 6, "cpu", flags, 0, romz=["Pong", "Pong"])
    th.set_training_stage(0)
    fp = np.zeros((4, 3))
    fp[1, 0] = 1
    th.local_network.set_fixed_path(fp)
    th.local_network.set_geopath(np.ones((4, 3)))
    seg = glob.store.layout.by_name["layer1.module0.weight"]
    frozen_before = glob.store.flat[seg.offset:seg.offset + seg.numel].detach().clone()
    head = glob.store.layout.by_name["policy.weight"]
    head_before = glob.store.flat[head.offset:head.offset + head.numel].detach().clone()
    scores = {}
    n = th.process(None, 0, score_set_ops=scores)
    assert 1 <= n <= 20
    assert torch.equal(glob.store.flat[seg.offset:seg.offset + seg.numel], frozen_before)
    assert not torch.equal(glob.store.flat[head.offset:head.offset + head.numel], head_before)


def _write_idx(path, arr):
    hdr = bytes([0, 0, 8, arr.ndim]) + np.asarray(arr.shape, dtype=">u4").tobytes()
    with gzip.open(path + ".gz", "wb") as f:
        f.write(hdr + arr.astype(np.uint8).tobytes())


def test_input_data_idx_and_synthetic(tmp_path):
    rng = np.random.RandomState(0)
    tx, ty = rng.randint(0, 256, (30, 28, 28)), rng.randint(0, 10, 30)
    _write_idx(str(tmp_path / "train-images-idx3-ubyte"), tx)
    _write_idx(str(tmp_path / "train-labels-idx1-ubyte"), ty)
    _write_idx(str(tmp_path / "t10k-images-idx3-ubyte"), tx[:7])
    _write_idx(str(tmp_path / "t10k-labels-idx1-ubyte"), ty[:7])
    ds = read_data_sets(str(tmp_path), one_hot=True, validation_size=10)
    assert ds.train.num_examples == 20 and ds.validation.num_examples == 10 and ds.test.num_examples == 7
    assert np.allclose(ds.test.images[0], tx[0].reshape(-1) / 255.0)
    assert np.array_equal(ds.test.labels.argmax(1), ty[:7])
    xb, yb = ds.train.next_batch(25)
    assert xb.shape == (25, 784) and yb.shape == (25, 10) and ds.train.epochs_completed == 1
    syn = read_data_sets(str(tmp_path / "missing"), synthetic_size=(120, 30))
    assert syn.train.images.shape[1] == 784 and syn.test.num_examples == 30
    assert set(np.unique(syn.train.labels)) <= set(range(10))
