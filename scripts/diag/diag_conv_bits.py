"""Per-layer forward outputs and ReLU bits: fast (compile-time geometry) vs generic conv kernels."""
import sys
import torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_hip_kernels import small_pixel_cfg, random_masks, make_model, DEV   # noqa: E402
from pathnet_gym_amd.ops import _lib   # noqa: E402

cfg = small_pixel_cfg()
P, E, T = 4, 16, 2
masks = random_masks(P, cfg.L, cfg.M, cfg.N, seed=9)
m = make_model(cfg, P, masks, seed=11)
g = torch.Generator(device="cpu").manual_seed(4)
obs = torch.stack([torch.randint(0, 256, (P * E, 160, 120, 4), generator=g, dtype=torch.uint8)
                   for _ in range(T)]).reshape(T, P * E, -1).to(DEV)
lib = _lib.lib()
hp = m.hip
for f16 in (0, 1):
    lib.fast_conv_set_f16_fwd(f16)
    res = {}
    for fast in (False, True):
        _lib.USE_FAST = fast
        acts, bits = [], []
        for l, gm in enumerate(hp.geoms):
            acts.append(torch.zeros(T, P * E, gm.out_feat, dtype=torch.bfloat16, device=DEV))
            b, r = hp.alloc_bits(l, T, P * E)
            b.fill_(0xAB)
            bits.append((b, r))
        for t in range(T):
            x = obs
            for l in range(len(hp.geoms)):
                hp.layer_fwd(l, x, acts[l], bits[l][0], P, E, 1, t, bits[l][1])
                x = acts[l]
        torch.cuda.synchronize()
        res[fast] = (acts, bits)
    _lib.USE_FAST = True
    for l in range(3):
        a0, a1 = res[False][0][l], res[True][0][l]
        b0, b1 = res[False][1][l][0], res[True][1][l][0]
        nb = int((b0 != b1).sum())
        print(f"f16={f16} layer {l}: acts equal {torch.equal(a0, a1)} max|d| {float((a0.float() - a1.float()).abs().max()):.4g}"
              f"  bits bytes {b0.numel()} mismatched {nb}", flush=True)
        if nb:
            idx = (b0 != b1).reshape(-1).nonzero()[:8].reshape(-1).tolist()
            print("   first mismatches", idx, b0.reshape(-1)[idx].tolist(), b1.reshape(-1)[idx].tolist())
lib.fast_conv_set_f16_fwd(1)
