"""Backward of every trunk layer at the bench shape under two grid settings (the round-5 whole-round grids vs the
earlier by-work grids), on the same data in one process: the weight gradients and input gradients must agree to
the fp32 summation-order level.  A grid partition that drops or repeats work shows up as an O(1) difference.

    python scripts/diag/grid_consistency.py --paths 64
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from pathnet_gym_amd.algo.trainer import PathNetTrainer  # noqa: E402
from pathnet_gym_amd.config import preset  # noqa: E402
from pathnet_gym_amd.ops import _lib  # noqa: E402

NEW = "x3_wg_auto=1,x3_wg_target=1536,x3_wg2_target=512,x3_dg3_target=512,x3_wg3_target=256,x3_fcw_target=1024,x3_dg_target=512"
OLD = "x3_wg_auto=0,x3_wg_target=1536,x3_wg2_target=0,x3_dg3_target=0,x3_wg3_target=512,x3_fcw_target=2048,x3_dg_target=2048"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--paths", type=int, default=64)
    ap.add_argument("--a", default=NEW)
    ap.add_argument("--b", default=OLD)
    a = ap.parse_args()
    cfg = preset("pong")
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = a.paths, 32, 20
    cfg.compute_dtype = "fp32x"
    cfg.frame_ring = True
    cfg.ga.backend = "device"
    tr = PathNetTrainer(cfg, device="cuda")
    for _ in range(3):
        tr.update()
    tr.flush()
    torch.cuda.synchronize()
    e, hp = tr.engine, tr.engine.hip
    P, E, T = e.P, e.E, e.T
    lib = _lib.lib()

    def setopt(arm):
        for kv in arm.split(","):
            k, v = kv.split("=")
            getattr(lib, "fast_conv_set_" + k)(int(v))

    segs = tr.model.store.layout.segments
    L = len(hp.geoms)
    out = []
    for l in range(L - 1, -1, -1):
        res = []
        for arm in (a.b, a.a):
            setopt(arm)
            g = torch.zeros_like(e.grad_flat)
            if l == 0:
                hp.ring_wgrad(e.frames, e.fc, e.grads[0], e.bits[0], g, P, E, T, e.bits_rows[0], rbase=e.rbase)
                dx = None
            else:
                hp.layer_bwd(l, e.acts[l - 1], e.grads[l], e.bits[l], g, e.grads[l - 1], P, E, T, e.bits_rows[l])
                dx = e.grads[l - 1].float().clone()
            torch.cuda.synchronize()
            res.append((g, dx))
        (gb, db), (ga, da) = res
        idx = [s for s in segs if s.layer == l]
        lo, hi = min(s.offset for s in idx), max(s.offset + s.numel for s in idx)
        wb, wa = gb[lo:hi].double(), ga[lo:hi].double()
        rec = {"layer": l, "wgrad_rel": float((wa - wb).abs().max() / wb.abs().max().clamp_min(1e-30)),
               "wgrad_norm": float(wb.norm()), "outside_layer_nonzero": bool(ga[:lo].any() or ga[hi:].any())}
        if db is not None:
            rec["dgrad_rel"] = float((da.double() - db.double()).abs().max() / db.double().abs().max().clamp_min(1e-30))
        out.append(rec)
        print(json.dumps(rec), flush=True)
    bad = [r for r in out if r["wgrad_rel"] > 1e-4 or r.get("dgrad_rel", 0) > 1e-4]
    print(json.dumps({"paths": a.paths, "ok": not bad, "layers": out}))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
