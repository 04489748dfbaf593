#!/usr/bin/env python3
"""Where does the fp32x LSTM network's gradient error come from?  (GPU diagnostic.)

Runs the tests/test_x3_engine.py eager LSTM fixture (reference preset, fp32x, small shape) and recomputes the whole
update in float64 and in plain fp32 with every layer output's gradient retained, then prints, layer by layer, the
relative error of the engine's stored forward values (trunk outputs, LSTM h) and of its output gradients
(engine.grads[l], written by layer l+1's dgrad / the LSTM backward) against the float64 truth, beside the plain fp32
oracle's error on the same quantity:

    python scripts/diag/x3_lstm_diag.py --task Pong
"""
from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

DEV = "cuda"


def rel(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float((a - b).norm() / (b.norm() + 1e-300))


def pair16(h, scale=1.0):
    """The fp16 pair (hi + lo, fp16 subnormals included) of h * scale, unscaled, as an identity-gradient rounding."""
    v = (h.detach() * scale).float()
    hi = v.half().float()
    lo = (v - hi).half().float()
    return h + ((hi.to(h.dtype) + lo.to(h.dtype)) / scale - h).detach()


def oracle(tr, eng, dtype, act_round=None):
    """Whole-update autograd in dtype; returns per-layer outputs / output gradients, the LSTM h's, the grad flat."""
    from pathnet_gym_amd.algo.a2c_math import a2c_loss, nstep_returns
    from pathnet_gym_amd.models.pathnet import ParamStore, heads_ref, lstm_cell_ref
    cfg = tr.cfg
    T, B = eng.T, eng.B
    a2c = cfg.a2c
    flat = tr.model.store.flat.detach().clone().to(dtype).requires_grad_(True)
    st = ParamStore(cfg.net, DEV, flat=flat)
    x = eng.obs_stacks().reshape((T + 1) * B, 160, 120, 4).to(dtype) / 255.0
    mask = tr.model.mask.repeat_interleave(eng.E, 0).repeat(T + 1, 1, 1).to(dtype)
    M = cfg.net.M
    h = x
    outs, masks0, fcm = [], None, {}
    for l, spec in enumerate(cfg.net.layers):
        li = st.layout.layer_info[l]
        W, b = st.W(l), st.b(l)
        m = mask[:, l, :]
        cout = li["cout"]
        if spec.kind == "conv":
            k = spec.kernel
            Wc = W.reshape(M, k, k, li["cin"], cout).permute(0, 4, 3, 1, 2).reshape(M * cout, li["cin"], k, k)
            y = F.conv2d(h.permute(0, 3, 1, 2), Wc, b.reshape(-1), stride=spec.stride)
            if l == 0:
                masks0 = (y.detach() > 0).view(h.shape[0], M, cout, y.shape[2], y.shape[3]) * m[:, :, None, None, None]
            y = F.relu(y).view(h.shape[0], M, cout, y.shape[2], y.shape[3]) * m[:, :, None, None, None]
            h = y.sum(1).permute(0, 2, 3, 1)
        else:
            pre = torch.einsum("bk,mkc->bmc", h.reshape(h.shape[0], -1), W) + b[None]
            fcm[l] = (pre.detach() > 0, pre.detach())
            h = (F.relu(pre) * m[:, :, None]).sum(1)
        if act_round is not None and l < cfg.net.L - 1:
            h = pair16(h, act_round)               # the engine's storage of a layer output between layers
        h.retain_grad()
        outs.append(h)
    feat = outs[-1].reshape(T + 1, B, -1)
    if cfg.net.trunk_scale == "M":
        feat = feat / M
    k, bb = st.lstm()
    hh, c = eng.hst[0].to(dtype), eng.cst[0].to(dtype)
    hs = []
    for t in range(T + 1):
        if t > 0:
            keep = (1.0 - eng.dones[t - 1].to(dtype))[:, None]
            hh, c = hh * keep, c * keep
        hh, c = lstm_cell_ref(feat[t], hh, c, k, bb)
        hs.append(hh)
    hcat = torch.stack(hs).reshape((T + 1) * B, -1)
    logits, values = heads_ref(st, hcat, tr.model.task)
    R, adv = nstep_returns(eng.rewards, eng.values[:T], eng.dones.bool(), eng.values[T], a2c.gamma,
                           a2c.gae_lambda, a2c.reward_clip)
    loss, _, _, _ = a2c_loss(logits[:T * B], values[:T * B], eng.actions[:T].reshape(-1).long(),
                             R.reshape(-1).to(dtype), adv.reshape(-1).to(dtype), a2c.entropy_beta, a2c.value_coef,
                             torch.full((T * B,), eng.weight, device=DEV, dtype=dtype))
    loss.backward(retain_graph=True)

    def from_layer(l, G):
        """dtype weight gradients of layers <= l given the output gradient G [T*B, feat] of layer l."""
        gz = torch.zeros((T + 1) * B, G.shape[-1], dtype=dtype, device=DEV)
        gz[:T * B] = G.to(dtype)
        return torch.autograd.grad(outs[l], flat, grad_outputs=gz.view_as(outs[l]), retain_graph=True)[0]

    return dict(from_layer=from_layer, acts=[o.detach().reshape((T + 1) * B, -1) for o in outs],
                grads=[o.grad.reshape((T + 1) * B, -1)[:T * B] for o in outs], h=hcat.detach(), flat=flat.grad,
                x=x.detach(), masks0=masks0, fcm=fcm)


def conv1_wgrad64(tr, eng, o64, G0):
    """float64 conv1 weight gradient of a given conv1 output gradient G0 [T*B, Ho*Wo*Cout] under the float64
    forward's ReLU masks, in the engine's flat layout (weights only)."""
    cfg = tr.cfg
    T, B = eng.T, eng.B
    spec = cfg.net.layers[0]
    li = tr.model.store.layout.layer_info[0]
    M, cout, cin, k = cfg.net.M, li["cout"], li["cin"], spec.kernel
    m = o64["masks0"][:T * B]                                       # [TB, M, cout, Ho, Wo]
    Ho, Wo = m.shape[3], m.shape[4]
    g = G0.double().view(T * B, Ho, Wo, cout).permute(0, 3, 1, 2)
    xn = o64["x"][:T * B].permute(0, 3, 1, 2)
    out = []
    for j in range(M):
        dW = torch.nn.grad.conv2d_weight(xn, (cout, cin, k, k), g * m[:, j], stride=spec.stride)
        out.append(dW.permute(2, 3, 1, 0).reshape(-1, cout))
    return torch.stack(out)                                         # [M, K, cout]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--task", default="Pong")
    ap.add_argument("--ring", type=int, default=1)
    a = ap.parse_args()
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
    from test_x3_engine import layer_errors, masks_with_edges
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    from pathnet_gym_amd.config import preset
    from pathnet_gym_amd.ops.pathnet_ops import x2_value
    cfg = preset("reference")
    cfg.tasks = [a.task] + [t for t in cfg.tasks if t != a.task]
    cfg.env = a.task
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 3, 16, 4
    cfg.compute_dtype = "fp32x"
    cfg.frame_ring = bool(a.ring)
    cfg.use_graph = False
    cfg.ga.backend = "device"
    tr = PathNetTrainer(cfg, device=DEV)
    eng = tr.engine
    tr.env.max_episode_steps = 5
    tr.update()
    tr.flush()
    tr.model.set_paths(masks_with_edges(3, cfg.net.L, cfg.net.M, cfg.net.N, seed=2))
    eng.rollout_backward()
    torch.cuda.synchronize()
    T, B = eng.T, eng.B
    o64, o32 = oracle(tr, eng, torch.float64), oracle(tr, eng, torch.float32)
    print(f"{a.task} ring={a.ring}: relative error vs float64 (engine | plain fp32)")
    for l in range(len(eng.acts)):
        act = eng.acts[l]
        av = (x2_value(act) if act.dtype == torch.float16 else act.float()).reshape((T + 1) * B, -1)
        print(f"  layer {l} output    {rel(av, o64['acts'][l]):.2e} | {rel(o32['acts'][l], o64['acts'][l]):.2e}")
    print(f"  lstm h            {rel(eng.hst[1:T + 2].reshape((T + 1) * B, -1), o64['h']):.2e} | "
          f"{rel(o32['h'], o64['h']):.2e}")
    for l in range(len(eng.grads) - 1, -1, -1):
        print(f"  layer {l} out grad  {rel(eng.grads[l].float(), o64['grads'][l]):.2e} | "
              f"{rel(o32['grads'][l], o64['grads'][l]):.2e}   amax engine {float(tr.model.hip.gamax[l]):.3e} "
              f"true {float(o64['grads'][l].abs().max()):.3e}")
    st = tr.model.store
    li = st.layout.layer_info[0]
    W_of = lambda fl: fl.as_strided((li["M"], li["K"], li["cout"]), (li["chunk"], li["cout"], 1), li["offset"])
    w_eng, w64, w32 = W_of(eng.grad_flat), W_of(o64["flat"]), W_of(o32["flat"])
    r_eng = conv1_wgrad64(tr, eng, o64, eng.grads[0].float())
    r_64 = conv1_wgrad64(tr, eng, o64, o64["grads"][0])
    print(f"  conv1 weights: engine vs float64 truth {rel(w_eng, w64):.2e}, plain fp32 {rel(w32, w64):.2e};"
          f" float64 wgrad of the ENGINE's G0 vs truth {rel(r_eng, w64):.2e}, engine vs that {rel(w_eng, r_eng):.2e};"
          f" float64 wgrad of the truth's G0 vs truth {rel(r_64, w64):.2e}")
    e = layer_errors(tr, eng.grad_flat, o64["flat"])
    e32 = layer_errors(tr, o32["flat"], o64["flat"])
    print("  weight grads      ", {k: f"{v:.2e} | {e32[k]:.2e}" for k, v in e.items()})
    for l in range(len(eng.grads) - 1, -1, -1):
        gl = o64["from_layer"](l, eng.grads[l].float())
        el = layer_errors(tr, gl, o64["flat"])
        print(f"  float64 backward from the ENGINE's layer {l} output gradient: ",
              {k: f"{v:.2e}" for k, v in el.items() if isinstance(k, int) and k <= l})
    # the top fc layer's input gradient under the ENGINE's ReLU bits (bits[l]: [slot][row][Cout/16] int16) in float64
    l = len(eng.grads) - 1
    g3 = tr.model.hip.geoms[l]
    if g3.kind == "fc":
        li = st.layout.layer_info[l]
        Wl = st.flat.double().as_strided((li["M"], li["K"], li["cout"]), (li["chunk"], li["cout"], 1), li["offset"])
        bw = eng.bits[l][:, :T * B].to(torch.int32) & 0xFFFF            # [slots, rows, Cout/16]
        sh = torch.arange(16, device=DEV)
        ebits = ((bw[..., None] >> sh) & 1).reshape(bw.shape[0], T * B, -1).bool()   # [slots, rows, Cout]
        act_idx, act_cnt = tr.model.act_idx, tr.model.act_cnt
        P, E = eng.P, eng.E
        G3 = eng.grads[l].double()
        G2 = torch.zeros(T * B, li["K"], dtype=torch.float64, device=DEV)
        m64, pre64 = o64["fcm"][l]
        flips, near = 0, []
        rows = torch.arange(T * B, device=DEV)
        pidx = (rows % B) // E
        for p in range(P):
            rs = rows[pidx == p]
            for j in range(int(act_cnt.view(P, -1)[p, l])):
                mod = int(act_idx.view(P, tr.cfg.net.L, -1)[p, l, j])
                mk = ebits[j, rs]
                G2[rs] += (G3[rs] * mk) @ Wl[mod].T
                tm = m64[rs, mod]
                d = mk != tm
                flips += int(d.sum())
                if d.any():
                    near.append(float(pre64[rs, mod][d].abs().max()))
        print(f"  layer {l} ReLU bits: engine vs float64 masks differ at {flips} elements (max |pre| there "
              f"{max(near) if near else 0:.2e}); float64 input gradient under the ENGINE's bits vs engine "
              f"{rel(eng.grads[l - 1], G2):.2e}, vs truth {rel(G2, o64['grads'][l - 1]):.2e}")
        dG = eng.grads[l - 1].double() - G2
        for p in range(P):
            rs = rows[pidx == p]
            print(f"    path {p}: {int(act_cnt.view(P, -1)[p, l])} slots, rel err {rel(eng.grads[l - 1][rs], G2[rs]):.2e}")
        rn = dG.norm(dim=1) / G2.norm(dim=1).clamp_min(1e-300)
        top = torch.topk(rn, 5)
        print("    worst rows (row, rel):", [(int(i), f"{float(v):.2e}") for v, i in zip(top.values, top.indices)])
        cn = dG.norm(dim=0) / G2.norm(dim=0).clamp_min(1e-300)
        top = torch.topk(cn, 5)
        print("    worst columns (k, rel):", [(int(i), f"{float(v):.2e}") for v, i in zip(top.values, top.indices)])
        print(f"    error coherence: |sum over rows of dG| / sum of |dG| rows = "
              f"{float(dG.sum(0).norm() / dG.norm(dim=1).sum()):.3f}; same for G2 {float(G2.sum(0).norm() / G2.norm(dim=1).sum()):.3f}")
        gl = o64["from_layer"](l - 1, G2)
        print("  float64 backward from that input gradient:",
              {k: f"{v:.2e}" for k, v in layer_errors(tr, gl, o64["flat"]).items() if isinstance(k, int) and k < l})

        def pair(x, scale, kind=torch.float16, pieces=2):
            v = x * scale
            out = torch.zeros_like(v)
            for _ in range(pieces):
                piece = v.float().to(kind).double()
                out += piece
                v = v - piece
            return out / scale

        def g16s(x):
            am = float(x.abs().max())
            return 2.0 ** (13 - int(torch.tensor(am).log2().floor())) if am > 0 else 1.0

        variants = {"W fp16 pair (x2^8), G exact": (lambda w: pair(w, 256.0), lambda g: g),
                    "W exact, G fp16 pair (G16)": (lambda w: w, lambda g: pair(g, g16s(g))),
                    "both pairs (the engine)": (lambda w: pair(w, 256.0), lambda g: pair(g, g16s(g))),
                    "W fp16 triple, G pair": (lambda w: pair(w, 256.0, pieces=3), lambda g: pair(g, g16s(g))),
                    "W bf16 triple, G pair": (lambda w: pair(w, 1.0, torch.bfloat16, 3), lambda g: pair(g, g16s(g)))}
        G32 = torch.zeros(T * B, li["K"], dtype=torch.float32, device=DEV)
        G32e = torch.zeros(T * B, li["K"], dtype=torch.float32, device=DEV)
        for p in range(P):
            rs = rows[pidx == p]
            mods = [int(act_idx.view(P, tr.cfg.net.L, -1)[p, l, j]) for j in range(int(act_cnt.view(P, -1)[p, l]))]
            for j, mod in enumerate(mods):
                G32[rs] += (G3[rs] * ebits[j, rs]).float() @ Wl[mod].float().T
            # one fp32 GEMM over (slot, column) jointly, as autograd's einsum backward does
            Gcat = torch.cat([(G3[rs] * ebits[j, rs]).float() for j in range(len(mods))], 1)
            Wcat = torch.cat([Wl[mod].float() for mod in mods], 1)
            G32e[rs] = Gcat @ Wcat.T
        # the engine's own operands (Gm fp16 planes, WcT fp16 pieces) multiplied EXACTLY: what the MFMA chain should
        # return; engine - that = the kernel's accumulation error alone
        hp = tr.model.hip
        gmv = hp._gm.view(torch.float16).view(2, hp.M, -1, 256).double()
        wct = hp.WcT[l].double()
        gsc = 2.0 ** (13 - int(torch.floor(torch.log2(hp.gamax[l].double()))))
        ideal = torch.zeros_like(G2)
        for p in range(P):
            rs = rows[pidx == p]
            for j in range(int(act_cnt.view(P, -1)[p, l])):
                mod = int(act_idx.view(P, tr.cfg.net.L, -1)[p, l, j])
                gh, gl = gmv[0, j, rs], gmv[1, j, rs]
                wh, wl = wct[0, mod, :li["K"]], wct[1, mod, :li["K"]]
                ideal[rs] += gh @ wh.T + gh @ wl.T + gl @ wh.T
        ideal /= gsc * 256.0
        d = eng.grads[l - 1].double() - ideal
        print(f"  fc input gradient: engine vs exact products of its own operands {rel(eng.grads[l - 1], ideal):.2e}"
              f" (operands vs truth {rel(ideal, G2):.2e}); <d, ideal>/<ideal, ideal> = "
              f"{float((d * ideal).sum() / (ideal * ideal).sum()):.3e}; mean d*sign(ideal)/mean|d| = "
              f"{float((d * ideal.sign()).mean() / d.abs().mean()):.3f}; mean d / mean|d| = "
              f"{float(d.mean() / d.abs().mean()):.3f}; d vs |ideal| correlation "
              f"{float(torch.corrcoef(torch.stack([d.flatten(), ideal.abs().flatten()]))[0, 1]):.3f}")
        gl_ = o64["from_layer"](l - 1, ideal)
        print("  float64 backward from the exact products:",
              {k: f"{v:.2e}" for k, v in layer_errors(tr, gl_, o64["flat"]).items() if isinstance(k, int) and k < l})
        for name, Gv in (("plain fp32, per-slot GEMMs summed", G32), ("plain fp32, one GEMM over slots", G32e)):
            gl = o64["from_layer"](l - 1, Gv.double())
            print(f"  fc input gradient {name:34s}: vs exact {rel(Gv, G2):.2e}; backward from it:",
                  {k: f"{v:.2e}" for k, v in layer_errors(tr, gl, o64["flat"]).items() if isinstance(k, int) and k < l})
        for name, (fw, fg) in variants.items():
            Gv = torch.zeros_like(G2)
            for p in range(P):
                rs = rows[pidx == p]
                for j in range(int(act_cnt.view(P, -1)[p, l])):
                    mod = int(act_idx.view(P, tr.cfg.net.L, -1)[p, l, j])
                    Gv[rs] += fg(G3[rs] * ebits[j, rs]) @ fw(Wl[mod]).T
            gl = o64["from_layer"](l - 1, Gv)
            print(f"  fc input gradient with {name:32s}: vs exact {rel(Gv, G2):.2e}; backward from it:",
                  {k: f"{v:.2e}" for k, v in layer_errors(tr, gl, o64["flat"]).items() if isinstance(k, int) and k < l})
    # the trunk backward again from the same top gradient, with the weights as three fp16 pieces in the input
    # gradients (csrc/trunk_x3.hip X3_DG_W3) and as the default pair
    from pathnet_gym_amd.ops import _lib
    lib = _lib.lib()
    keep = eng.grad_flat.clone()
    for w3, fold in ((0, 0), (1, 0), (0, 1), (0, 2)):
        lib.fast_conv_set_x3_dg_w3(w3)
        lib.fast_conv_set_x3_dg_fold(fold)
        eng.grad_flat.zero_()
        eng._layer_bwd_all(T, 0)
        torch.cuda.synchronize()
        e = layer_errors(tr, eng.grad_flat, o64["flat"])
        print(f"  trunk backward, weights as {3 if w3 else 2} fp16 pieces, fold {fold}:",
              {k: f"{v:.2e}" for k, v in e.items() if isinstance(k, int)})
    lib.fast_conv_set_x3_dg_w3(0)
    lib.fast_conv_set_x3_dg_fold(0)
    eng.grad_flat.copy_(keep)
    for sc in (1.0, 256.0):
        r = oracle(tr, eng, torch.float64, act_round=sc)
        er = layer_errors(tr, r["flat"], o64["flat"])
        print(f"  float64 with layer outputs stored as fp16 pairs of A * {sc:g}: ",
              {k: f"{v:.2e}" for k, v in er.items()})


if __name__ == "__main__":
    main()
