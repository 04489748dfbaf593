"""fc1 forward (module-major, k split into parts) at the bench shape under two part counts, same inputs: the
activations must agree to fp32 summation-order level and the ReLU bits must agree except where a pre-activation sits
within rounding of zero.

    python scripts/diag/fc_ks_consistency.py --paths 64 --a 2 --b 3
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--paths", type=int, default=64)
    ap.add_argument("--a", type=int, default=2)
    ap.add_argument("--b", type=int, default=3)
    ap.add_argument("--layer", type=int, default=3)
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
    lib = _lib.lib()
    l = a.layer
    outs = []
    for ks in (a.a, a.b):
        lib.fast_conv_set_x3_fc_ks_parts(ks)
        hp.layer_fwd(l, e.acts[l - 1], e.acts[l], e.bits[l], e.P, e.E, 1, 3, e.bits_rows[l])
        torch.cuda.synchronize()
        outs.append((e.acts[l][3].double().clone(), e.bits[l].clone()))
    lib.fast_conv_set_x3_fc_ks_parts(0)
    (ya, ba), (yb, bb) = outs
    rel = float((ya - yb).abs().max() / ya.abs().max().clamp_min(1e-30))
    nbits = int((ba != bb).sum())
    rec = {"paths": a.paths, "ks": [a.a, a.b], "act_rel": rel, "bits_diff_bytes": nbits, "act_norm": float(ya.norm())}
    print(json.dumps(rec))
    sys.exit(0 if rel < 1e-5 else 1)


if __name__ == "__main__":
    main()
