#!/usr/bin/env python3
"""Pipelined device-GA mode WITHOUT per-update syncs: keep a device-side history of the reduced
[fitness | counters] (stream-ordered copies right after each exchange) and compare it at the end with
what the pipeline's host readback collected for the same updates."""
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
    nup = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    mode = sys.argv[2] if len(sys.argv) > 2 else "plain"
    cfg = preset("pong")
    cfg.use_graph = mode != "eager"
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 16, 16, 5
    cfg.ga.backend = "device"
    cfg.ga.concurrent_tournaments = 1
    tr = PathNetTrainer(cfg, device="cuda")
    comm = tr.comm
    P = comm.P_total
    hist = torch.zeros(nup + 2, P + 4, device="cuda")
    hist_cnt = torch.zeros(nup + 2, 4, device="cuda")
    collected = []
    orig_ex, orig_col = comm.exchange_async, comm.collect
    k = {"n": 0}

    def ex(grad, fit, counters, extra=None):
        h = orig_ex(grad, fit, counters, extra=extra)
        hist[k["n"]].copy_(comm.small_dev)
        hist_cnt[k["n"]].copy_(counters)
        k["n"] += 1
        return h

    def col(handle):
        f, c, s = orig_col(handle)
        collected.append(np.concatenate([f, c]))
        return f, c, s
    comm.exchange_async, comm.collect = ex, col
    eng = tr.engine
    rb, os_ = eng.rollout_backward, eng.optimizer_step

    def barrier():
        e = torch.cuda.Event()
        e.record()
        torch.cuda.current_stream().wait_event(e)

    def rb2():
        rb()
        if mode == "sync_rollout":
            torch.cuda.synchronize()
        if mode == "barrier":
            barrier()

    def os2(lr, skip=False):
        os_(lr, skip)
        if mode == "sync_opt":
            torch.cuda.synchronize()
        if mode == "barrier":
            barrier()
    eng.rollout_backward, eng.optimizer_step = rb2, os2
    t0 = time.time()
    for i in range(nup):
        tr.update()
        if i % 1000 == 0:
            print(json.dumps({"update": i, "t": round(time.time() - t0, 1)}), flush=True)
    tr.flush()
    torch.cuda.synchronize()
    H = hist[:len(collected)].cpu().numpy()
    HC = hist_cnt[:len(collected)].cpu().numpy()
    C = np.stack(collected)
    bad_dev = np.nonzero(np.abs(H[:, P + 2]) > 21 * np.maximum(H[:, P + 1], 1))[0]
    bad_col = np.nonzero(np.abs(C[:, P + 2]) > 21 * np.maximum(C[:, P + 1], 1))[0]
    diff = np.nonzero(np.any(H != C, axis=1))[0]
    out = {"mode": mode, "updates": len(collected), "bad_device": len(bad_dev), "bad_collected": len(bad_col),
           "device_vs_collected_differ": len(diff), "first_bad_dev": bad_dev[:5].tolist(),
           "first_bad_col": bad_col[:5].tolist(), "first_diff": diff[:5].tolist()}
    for j in list(diff[:3]):
        out[f"u{j}"] = {"dev": H[j, P:].tolist(), "col": C[j, P:].tolist(), "counters_buf": HC[j].tolist(),
                        "dev_fit": H[j, :4].tolist(), "col_fit": C[j, :4].tolist()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
