"""Why the reference preset's trunk kernels run slower than the Pong preset's on the SAME geometry (profiles/r6/
kwin_reference_preset.md vs kwin_p64_window0.md): time the conv1 ring forward and the conv3 backward of both engines
interleaved in one process, then again with the Pong engine's frames copied into the reference engine's ring."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from pathnet_gym_amd import _build  # noqa: E402
_build.build()
from pathnet_gym_amd.algo.trainer import PathNetTrainer  # noqa: E402
from pathnet_gym_amd.config import preset  # noqa: E402


def make(name):
    cfg = preset(name)
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 64, 32, 20
    cfg.compute_dtype, cfg.frame_ring, cfg.ga.backend = "fp32x", True, "device"
    cfg.ga.concurrent_tournaments = 4
    tr = PathNetTrainer(cfg, device="cuda")
    for _ in range(3):
        tr.update()
    tr.flush()
    torch.cuda.synchronize()
    return tr


def timeit(fn, reps=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


trs = {"pong": make("pong"), "reference": make("reference")}


def kernels(tr):
    e, hp = tr.engine, tr.model.hip
    P, E, T = e.P, e.E, e.T
    scratch = torch.zeros_like(e.grad_flat)
    return {
        "conv1_fwd": lambda: hp.ring_fwd(e.frames, e.fc, e.acts[0], e.bits[0], P, E, 1, 3, e.bits_rows[0],
                                         rbase=e.rbase),
        "conv1_wgrad": lambda: hp.ring_wgrad(e.frames, e.fc, e.grads[0], e.bits[0], scratch, P, E, T, e.bits_rows[0],
                                             rbase=e.rbase),
        "conv3_bwd": lambda: hp.layer_bwd(2, e.acts[1], e.grads[2], e.bits[2], scratch, e.grads[1], P, E, T,
                                          e.bits_rows[2]),
    }


def stats(tr):
    e = tr.engine
    out = {"act_cnt_mean": [round(float(x), 3) for x in tr.model.act_cnt.float().mean(0).tolist()]}
    for l in range(3):
        out[f"relu_on_frac_l{l}"] = round(float((e.bits[l].float() != 0).float().mean()), 4)
        out[f"grad_abs_mean_l{l}"] = float(e.grads[l].float().abs().mean())
        out[f"act_abs_mean_l{l}"] = float(e.acts[l].float().abs().mean())
    out["frames_nonzero_frac"] = round(float((e.frames != 0).float().mean()), 4)
    return out


res = {k: {"stats": stats(tr)} for k, tr in trs.items()}
ks = {k: kernels(tr) for k, tr in trs.items()}
for rnd in range(5):
    for k in trs:
        for name, fn in ks[k].items():
            res[k].setdefault(name, []).append(timeit(fn))
for k in trs:
    for name in ks[k]:
        res[k][name + "_us"] = round(statistics.median(res[k].pop(name)), 1)
# the Pong engine's frames in the reference engine's ring (same layout: [B][2T][19200] uint8)
er, ep = trs["reference"].engine, trs["pong"].engine
if er.frames.shape == ep.frames.shape:
    er.frames.copy_(ep.frames)
    er.fc.copy_(ep.fc)
    t = [timeit(ks["reference"]["conv1_fwd"]) for _ in range(5)]
    res["reference"]["conv1_fwd_with_pong_frames_us"] = round(statistics.median(t), 1)
print(json.dumps(res, indent=1))
