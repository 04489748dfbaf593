#!/usr/bin/env python3
"""CPU emulation: how does the fp16-pair representation of a FIXED operand (the weights) propagate into the weight
gradients of the reference network (L=4 trunk + LSTM 256, A2C loss), compared with the rounding of per-sample
operands?  (Companion of scripts/diag/x3_lstm_diag.py, which measures the HIP engine itself on the GPU.)

Builds one synthetic update on CPU in float64 -- real synthetic-game frames (torch backend), the reference preset's
parameters, random paths, an A2C loss over T steps -- and recomputes the gradient with single stages rounded the way
csrc/trunk_x3.hip rounds them:

    python scripts/diag/x3_lstm_emul.py --game Pong
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

D = torch.float64


def rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-300))


def pieces(x, scale, kind=torch.float16, n=2):
    """x as the sum of n fp16 (or bf16) pieces of x * scale, unscaled (fp16 subnormals included)."""
    v = x * scale
    out = torch.zeros_like(v)
    for _ in range(n):
        p = v.float().to(kind).to(x.dtype)
        out = out + p
        v = v - p
    return out / scale


def g16(x):
    am = float(x.abs().max())
    return 2.0 ** (13 - int(np.floor(np.log2(am)))) if am > 0 else 1.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--game", default="Pong")
    ap.add_argument("--paths", type=int, default=3)
    ap.add_argument("--envs", type=int, default=16)
    ap.add_argument("--T", type=int, default=4)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    from pathnet_gym_amd.algo.a2c_math import a2c_loss, nstep_returns
    from pathnet_gym_amd.algo.ga import get_geopath
    from pathnet_gym_amd.config import preset
    from pathnet_gym_amd.envs.registry import make
    from pathnet_gym_amd.models.pathnet import ParamStore, heads_ref, lstm_cell_ref

    cfg = preset("reference")
    net = cfg.net
    P, E, T = a.paths, a.envs, a.T
    B = P * E
    torch.manual_seed(a.seed)
    env = make(a.game, num_envs=B, device="cpu", seed=a.seed, backend="torch")
    obs = env.reset()
    g = torch.Generator().manual_seed(a.seed)
    for _ in range(30):
        obs, _, _, _ = env.step(torch.randint(0, env.num_actions, (B,), generator=g))
    frames = []
    for _ in range(T + 1):
        frames.append(obs.clone())
        obs, _, _, _ = env.step(torch.randint(0, env.num_actions, (B,), generator=g))
    x = torch.stack(frames).reshape((T + 1) * B, 160, 120, 4).to(D) / 255.0
    rng = np.random.RandomState(a.seed)
    paths = np.stack([get_geopath(net.L, net.M, net.N, rng) for _ in range(P)])
    mask = torch.from_numpy(paths).to(D).repeat_interleave(E, 0).repeat(T + 1, 1, 1)
    store = ParamStore(net, "cpu", seed=a.seed)
    flat0 = store.flat.to(D)
    L, M = net.L, net.M
    A = net.num_actions
    actions = torch.randint(0, A, (T, B), generator=g)
    rewards = (torch.rand(T, B, generator=g) < 0.1).to(D) * torch.sign(torch.randn(T, B, generator=g)).to(D)
    dones = torch.zeros(T, B, dtype=torch.bool)

    def run(w_fwd=None, fc_dgrad=None):
        """Gradient of the update.  w_fwd(W, l): the weights the forward uses (rounding, identity gradient);
        fc_dgrad(Gm, W): the top fc layer's input-gradient product (custom autograd)."""
        flat = flat0.clone().requires_grad_(True)
        st = ParamStore(net, "cpu", flat=flat)
        h = x
        for l, spec in enumerate(net.layers):
            li = st.layout.layer_info[l]
            W, b = st.W(l), st.b(l)
            if w_fwd is not None:
                W = W + (w_fwd(W.detach(), l) - W.detach())
            m = mask[:, l, :]
            cout = li["cout"]
            if spec.kind == "conv":
                k = spec.kernel
                Wc = W.reshape(M, k, k, li["cin"], cout).permute(0, 4, 3, 1, 2).reshape(M * cout, li["cin"], k, k)
                y = F.conv2d(h.permute(0, 3, 1, 2), Wc, b.reshape(-1), stride=spec.stride)
                y = F.relu(y).view(h.shape[0], M, cout, y.shape[2], y.shape[3]) * m[:, :, None, None, None]
                h = y.sum(1).permute(0, 2, 3, 1)
            else:
                hf = h.reshape(h.shape[0], -1)
                if fc_dgrad is not None and l == L - 1:
                    h = _FC.apply(hf, W, b, m, fc_dgrad)
                else:
                    pre = torch.einsum("bk,mkc->bmc", hf, W) + b[None]
                    h = (F.relu(pre) * m[:, :, None]).sum(1)
        feat = h.reshape(T + 1, B, -1)
        kk, bb = st.lstm()
        hh = torch.zeros(B, kk.shape[1] // 4, dtype=D)
        c = torch.zeros_like(hh)
        hs = []
        for t in range(T + 1):
            hh, c = lstm_cell_ref(feat[t], hh, c, kk, bb)
            hs.append(hh)
        hcat = torch.stack(hs).reshape((T + 1) * B, -1)
        logits, values = heads_ref(st, hcat, 0)
        vals = values.detach().view(T + 1, B)
        R, adv = nstep_returns(rewards, vals[:T], dones, vals[T], cfg.a2c.gamma, cfg.a2c.gae_lambda,
                               cfg.a2c.reward_clip)
        loss, _, _, _ = a2c_loss(logits[:T * B], values[:T * B], actions.reshape(-1), R.reshape(-1),
                                 adv.reshape(-1), cfg.a2c.entropy_beta, cfg.a2c.value_coef,
                                 torch.full((T * B,), 1.0 / E, dtype=D))
        loss.backward()
        return flat.grad

    def errs(gv, gt):
        out = {}
        for s in store.layout.segments:
            key = s.layer if s.layer >= 0 else s.name.split(".")[0]
            out.setdefault(key, []).append((gv[s.offset:s.offset + s.numel], gt[s.offset:s.offset + s.numel]))
        return {k: f"{rel(torch.cat([u for u, _ in v]), torch.cat([w for _, w in v])):.2e}" for k, v in out.items()}

    truth = run()
    variants = {
        "fc dgrad: W fp16 pair (x2^8), G exact": lambda Gm, W: Gm @ pieces(W, 256.0).T,
        "fc dgrad: W exact, G fp16 pair (G16)": lambda Gm, W: pieces(Gm, g16(Gm)) @ W.T,
        "fc dgrad: both pairs, lo*lo dropped (engine)": lambda Gm, W: _mma3(Gm, W),
        "fc dgrad: G pair x W fp16 triple (4 MFMAs)": lambda Gm, W: _mma3(Gm, W, wtriple=True),
        "fc dgrad: G pair x W bf16 triple": lambda Gm, W: pieces(Gm, g16(Gm)) @ pieces(W, 1.0, torch.bfloat16, 3).T,
    }
    print(f"{a.game}: per-layer weight-gradient error vs float64, {P} paths x {E} envs, T={T}")
    for name, fn in variants.items():
        print(f"  {name:48s}", errs(run(fc_dgrad=fn), truth))
    print(f"  {'forward: all W fp16 pairs (x2^8)':48s}", errs(run(w_fwd=lambda W, l: pieces(W, 256.0)), truth))
    print(f"  {'forward: all W fp16 triples':48s}",
          errs(run(w_fwd=lambda W, l: pieces(W, 256.0, n=3)), truth))


def _mma3(Gm, W, wtriple=False):
    """hi*hi + hi*lo + lo*hi (+ hi*r: the weights' third fp16 piece) of G * 2^e and W * 2^8 pairs."""
    s = g16(Gm)
    gv = Gm * s
    gh = gv.float().half().to(gv.dtype)
    gl = (gv - gh).float().half().to(gv.dtype)
    wv = W * 256.0
    wh = wv.float().half().to(wv.dtype)
    wl = (wv - wh).float().half().to(wv.dtype)
    out = gh @ wh.T + gh @ wl.T + gl @ wh.T
    if wtriple:
        wr = (wv - wh - wl).float().half().to(wv.dtype)
        out = out + gh @ wr.T
    return out / (s * 256.0)


class _FC(torch.autograd.Function):
    """The masked module-sum fc layer whose input gradient is fn(masked G, W) per module (exact dW, db)."""

    @staticmethod
    def forward(ctx, hf, W, b, m, fn):
        pre = torch.einsum("bk,mkc->bmc", hf, W) + b[None]
        ctx.save_for_backward(hf, W, (pre > 0).to(hf.dtype) * m[:, :, None])
        ctx.fn = fn
        return (F.relu(pre) * m[:, :, None]).sum(1)

    @staticmethod
    def backward(ctx, gout):
        hf, W, r = ctx.saved_tensors
        dW = torch.zeros_like(W)
        db = torch.zeros(W.shape[0], W.shape[2], dtype=W.dtype)
        dhf = torch.zeros_like(hf)
        for j in range(W.shape[0]):
            Gm = gout * r[:, j]
            if not Gm.any():
                continue
            dW[j] = hf.T @ Gm
            db[j] = Gm.sum(0)
            dhf += ctx.fn(Gm, W[j])
        return dhf, dW, db, None, None


if __name__ == "__main__":
    main()
