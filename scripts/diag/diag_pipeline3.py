#!/usr/bin/env python3
"""Pipelined device-GA mode, no per-update host sync: per update, stream-ordered device snapshots of the
counters, an in-stream recomputation from eng.dones / eng.epret, and a few buffer statistics; dumped at the
end around the first implausible update."""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import numpy as np
    import torch
    from pathnet_gym_amd import _build
    _build.build()
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    from pathnet_gym_amd.config import preset
    from pathnet_gym_amd.envs.pong import EPRET
    nup = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    cfg = preset("pong")
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 16, 16, 5
    cfg.ga.backend = "device"
    cfg.ga.concurrent_tournaments = 1
    tr = PathNetTrainer(cfg, device="cuda")
    eng = tr.engine
    comm = tr.comm
    P = comm.P_total
    K = 12
    hist = torch.zeros(nup + 2, K, device="cuda")
    orig_ex = comm.exchange_async
    k = [0]

    def ex(grad, fit, counters, extra=None):
        h = orig_ex(grad, fit, counters, extra=extra)
        d = eng.dones
        dm = (d != 0)
        row = hist[k[0]]
        row[0:4].copy_(counters)
        row[4] = dm.sum()
        row[5] = (eng.epret * dm).sum()
        row[6] = d.max()
        row[7] = eng.epret.abs().max()
        row[8] = eng.env._st32[:, EPRET].abs().max()
        row[9] = eng.fitness.abs().max()
        row[10] = eng.stats[2]
        row[11] = eng.counters[1]
        k[0] += 1
        return h
    comm.exchange_async = ex
    orig_col = comm.collect

    def col(handle):
        f, c, st = orig_col(handle)
        c = np.where(np.isfinite(c) & (np.abs(c) < 1e12), c, 0.0)       # keep the host loop alive; hist keeps raw
        return f, c, st
    comm.collect = col
    t0 = time.time()
    for i in range(nup):
        tr.update()
        if i % 2000 == 0:
            print(json.dumps({"update": i, "t": round(time.time() - t0, 1)}), flush=True)
    tr.flush()
    torch.cuda.synchronize()
    H = hist[:k[0]].cpu().numpy()
    cnt, ret = H[:, 1], H[:, 2]
    bad = np.nonzero((np.abs(ret) > 21 * np.maximum(cnt, 1)) | (np.abs(cnt - H[:, 4]) > 0.5))[0]
    out = {"updates": int(k[0]), "bad": int(len(bad)), "first_bad": bad[:10].tolist()}
    if len(bad):
        b0 = int(bad[0])
        out["rows"] = {int(j): [float(x) for x in H[j]] for j in range(max(0, b0 - 2), min(len(H), b0 + 4))}
        out["bad_frac_after_onset"] = float(len(bad) / max(1, len(H) - b0))
        out["max_abs_epret_ever"] = float(H[:, 7].max())
        out["max_state_epret_ever"] = float(H[:, 8].max())
        out["max_done_ever"] = float(H[:, 6].max())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
