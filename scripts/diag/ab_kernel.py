"""Interleaved A/B timing of one engine kernel under two (or more) kernel-option settings, in ONE process on the
same data: a bench window per setting drifts by +-10 % between runs on one box (clock / thermal state), which
swamps a 5 % kernel change.  Example:

    python scripts/diag/ab_kernel.py --kernel ring_wgrad --opt x3_slab_pmap=0 --opt x3_slab_pmap=1
"""
import argparse
import json
import statistics
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from pathnet_gym_amd.algo.trainer import PathNetTrainer  # noqa: E402
from pathnet_gym_amd.config import preset  # noqa: E402
from pathnet_gym_amd.ops import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="ring_wgrad", choices=["ring_wgrad", "ring_fwd", "conv23_fwd", "layer_bwd", "layer_fwd", "fc_heads", "fc_then_heads"])
    ap.add_argument("--layer", type=int, default=1)
    ap.add_argument("--part", default=None, choices=["d", "w"], help="layer_bwd: input (d) or weight (w) gradient only")
    ap.add_argument("--opt", action="append", default=[],
                    help="one arm: name=value[,name=value...] (fast_conv_set_<name>); give every varied name in every arm")
    ap.add_argument("--paths", type=int, default=64)
    ap.add_argument("--preset", default="pong", help="pong, or reference (L=4 + LSTM: its population has paths of 5 "
                                                     "active modules in a layer)")
    ap.add_argument("--updates", type=int, default=2, help="updates before timing")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=6)
    a = ap.parse_args()
    cfg = preset(a.preset)
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = a.paths, 32, 20
    cfg.compute_dtype = "fp32x"
    cfg.frame_ring = True
    cfg.ga.backend = "device"
    tr = PathNetTrainer(cfg, device="cuda")
    for _ in range(a.updates):
        tr.update()
    tr.flush()
    torch.cuda.synchronize()
    e, hp = tr.engine, tr.engine.hip
    P, E, T = e.P, e.E, e.T
    scratch = torch.zeros_like(e.grad_flat)

    def run():
        if a.kernel == "ring_wgrad":
            hp.ring_wgrad(e.frames, e.fc, e.grads[0], e.bits[0], scratch, P, E, T, e.bits_rows[0], rbase=e.rbase)
        elif a.kernel == "ring_fwd":
            hp.ring_fwd(e.frames, e.fc, e.acts[0], e.bits[0], P, E, 1, 3, e.bits_rows[0], rbase=e.rbase)
        elif a.kernel == "conv23_fwd":
            hp.conv23_fwd(1, e.acts[0], e.acts[1], e.bits[1], e.bits_rows[1], e.acts[2], e.bits[2], e.bits_rows[2],
                          P, E, 1, 3)
        elif a.kernel == "fc_heads":
            L = len(hp.geoms)
            hp.fc_heads_fwd(e.acts[L - 2], e.acts[L - 1], e.bits[L - 1], e.bits_rows[L - 1], e.logits[3], e.values[3],
                            e.actions[3], e.seed, e.ctr, 3, T + 1, P, E, 3)
        elif a.kernel == "fc_then_heads":
            L = len(hp.geoms)
            hp.layer_fwd(L - 1, e.acts[L - 2], e.acts[L - 1], e.bits[L - 1], P, E, 1, 3, e.bits_rows[L - 1])
            hp.heads_fwd(e.acts[L - 1][3], e.logits[3], e.values[3], e.actions[3], e.seed, e.ctr, 3, T + 1)
        elif a.kernel == "layer_fwd":
            l = a.layer
            hp.layer_fwd(l, e.acts[l - 1], e.acts[l], e.bits[l], P, E, 1, 3, e.bits_rows[l])
        else:
            l = a.layer
            hp.layer_bwd(l, e.acts[l - 1], e.grads[l], e.bits[l], scratch, e.grads[l - 1], P, E, T, e.bits_rows[l],
                         part=a.part)

    arms = a.opt or ["none=0"]
    lib = _lib.lib()

    def setopt(arm):
        for kv in arm.split(","):
            k, v = kv.split("=")
            if k.startswith("py."):              # a HipPathNet attribute (e.g. py.fc_wgrad_gm_wgs=512)
                setattr(hp, k[3:], int(v))
            elif k != "none":
                getattr(lib, "fast_conv_set_" + k)(int(v))

    times = {kv: [] for kv in arms}
    for kv in arms:                       # one untimed pass per arm (first-touch / clock ramp)
        setopt(kv)
        run()
    for r in range(a.rounds):
        for kv in (arms if r % 2 == 0 else arms[::-1]):
            setopt(kv)
            run()
            torch.cuda.synchronize()
            s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.reps):
                run()
            t.record()
            torch.cuda.synchronize()
            times[kv].append(s.elapsed_time(t) / a.reps * 1e3)
    out = {kv: {"median_us": round(statistics.median(v), 1), "all_us": [round(x, 1) for x in v]} for kv, v in times.items()}
    cnt = tr.model.act_cnt.cpu()
    print(json.dumps({"kernel": a.kernel, "layer": a.layer, "part": a.part, "preset": a.preset, "paths": a.paths,
                      "active_max_per_layer": cnt.max(0).values.tolist(),
                      "paths_over_4_per_layer": (cnt > 4).sum(0).tolist(), "arms": out}))


if __name__ == "__main__":
    main()
