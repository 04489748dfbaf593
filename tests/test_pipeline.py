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
