"""PathNet super-network: flat module-major parameter store + reference forward.

Storage (MI355X-first, not the reference's one-TF-variable-per-tensor):
every parameter lives in ONE flat fp32 buffer.  Inside a PathNet layer the M
modules are stored module-major and each module is one contiguous chunk
``[W (K*Cout) | b (Cout)]``.  Consequences:

* the "active-path" gradient all-reduce packs whole modules as contiguous
  slices (``parallel/comm.py``);
* the multi-tensor RMSProp/clip kernel walks a segment table instead of
  ~2*L*M+8 separate tensors (``ops/optim.py``);
* freezing = excluding segments.

Logical tensors and their TF order (ref ``game_ac_network.py:317-347,397``)
are exposed as strided views; ``utils/checkpoint.py`` maps them to stable
names ``layer{i}.module{j}.weight`` etc.

The dense-masked forward here is the numerical ORACLE: every module is
computed, ReLU'd, multiplied by its mask and summed (exactly the reference
graph ``game_ac_network.py:182-201`` / ``:378-426``).  The HIP backend
(``models/acnet.py`` + ``ops/``) computes only active modules.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from ..config import PathNetConfig


@dataclass
class Segment:
    """One logical tensor inside the flat buffer (== one TF variable)."""
    name: str
    offset: int
    numel: int
    shape: Tuple[int, ...]
    layer: int = -1        # PathNet layer (-1 for heads / lstm)
    module: int = -1       # module index within the layer
    kind: str = ""         # "W" | "b"
    task: int = -1         # per-task head index (-1 shared)


class ParamLayout:
    """Offsets of every tensor in the flat buffer."""

    def __init__(self, cfg: PathNetConfig):
        self.cfg = cfg
        self.shapes = cfg.layer_shapes()
        self.segments: List[Segment] = []
        self.layer_info = []   # per layer: dict(offset, chunk, K, cout, M)
        off = 0
        M = cfg.M
        for l, (spec, (ins, outs, K, cin)) in enumerate(zip(cfg.layers, self.shapes)):
            cout = spec.out
            chunk = K * cout + cout
            self.layer_info.append(dict(offset=off, chunk=chunk, K=K, cout=cout, M=M, cin=cin,
                                        kind=spec.kind, kernel=spec.kernel, stride=spec.stride,
                                        in_shape=ins, out_shape=outs))
            for j in range(M):
                if spec.kind == "conv":
                    wshape = (spec.kernel, spec.kernel, cin, cout)
                else:
                    wshape = (K, cout)
                self.segments.append(Segment(f"layer{l}.module{j}.weight", off, K * cout, wshape, l, j, "W"))
                off += K * cout
                self.segments.append(Segment(f"layer{l}.module{j}.bias", off, cout, (cout,), l, j, "b"))
                off += cout
        self.trunk_numel = off
        feat = cfg.feature_dim
        self.lstm = None
        if cfg.use_lstm:
            H = cfg.lstm_size
            self.lstm = dict(kernel=off, bias=off + (feat + H) * 4 * H, H=H, din=feat)
            self.segments.append(Segment("lstm.kernel", off, (feat + H) * 4 * H, (feat + H, 4 * H)))
            off += (feat + H) * 4 * H
            self.segments.append(Segment("lstm.bias", off, 4 * H, (4 * H,)))
            off += 4 * H
            feat = H
        self.head_in = feat
        A = cfg.num_actions
        nheads = cfg.num_tasks if cfg.per_task_heads else 1
        self.heads = []
        for t in range(nheads):
            sfx = f".task{t}" if cfg.per_task_heads else ""
            h = {}
            self.segments.append(Segment(f"policy{sfx}.weight", off, feat * A, (feat, A), task=t if nheads > 1 else -1))
            h["pw"] = off; off += feat * A
            self.segments.append(Segment(f"policy{sfx}.bias", off, A, (A,), task=t if nheads > 1 else -1))
            h["pb"] = off; off += A
            self.segments.append(Segment(f"value{sfx}.weight", off, feat, (feat, 1), task=t if nheads > 1 else -1))
            h["vw"] = off; off += feat
            self.segments.append(Segment(f"value{sfx}.bias", off, 1, (1,), task=t if nheads > 1 else -1))
            h["vb"] = off; off += 1
            self.heads.append(h)
        self.numel = off
        self.by_name = {s.name: s for s in self.segments}

    def module_range(self, l: int, j: int) -> Tuple[int, int]:
        li = self.layer_info[l]
        s = li["offset"] + j * li["chunk"]
        return s, s + li["chunk"]


class ParamStore:
    """Flat parameter buffer + typed strided views."""

    def __init__(self, cfg: PathNetConfig, device="cpu", seed: int = 1, flat: Optional[torch.Tensor] = None):
        self.cfg = cfg
        self.layout = ParamLayout(cfg)
        self.device = torch.device(device)
        if flat is None:
            flat = torch.zeros(self.layout.numel, dtype=torch.float32)
            self._init(flat, seed)
            flat = flat.to(self.device)
        self.flat = flat

    # muupan init: U(-1/sqrt(fan_in), 1/sqrt(fan_in)) for W and b (game_ac_network.py:89-107);
    # LSTM kernel TF glorot_uniform default, bias zeros.
    def _init(self, flat: torch.Tensor, seed: int):
        g = torch.Generator().manual_seed(seed)
        for s in self.layout.segments:
            view = flat[s.offset:s.offset + s.numel]
            if s.name == "lstm.kernel":
                fan_in, fan_out = s.shape
                lim = math.sqrt(6.0 / (fan_in + fan_out))
                view.uniform_(-lim, lim, generator=g)
            elif s.name == "lstm.bias":
                view.zero_()
            else:
                if s.layer >= 0:
                    fan_in = self.layout.layer_info[s.layer]["K"]
                else:
                    base = s.name.split(".")[0]
                    fan_in = self.layout.head_in
                d = 1.0 / math.sqrt(fan_in)
                view.uniform_(-d, d, generator=g)

    # ---- views ----
    def W(self, l: int) -> torch.Tensor:
        """[M, K, Cout] strided view of layer l weights."""
        li = self.layout.layer_info[l]
        return self.flat.as_strided((li["M"], li["K"], li["cout"]), (li["chunk"], li["cout"], 1), li["offset"])

    def b(self, l: int) -> torch.Tensor:
        li = self.layout.layer_info[l]
        return self.flat.as_strided((li["M"], li["cout"]), (li["chunk"], 1), li["offset"] + li["K"] * li["cout"])

    def head(self, task: int = 0):
        h = self.layout.heads[task if self.cfg.per_task_heads else 0]
        F_ = self.layout.head_in
        A = self.cfg.num_actions
        pw = self.flat[h["pw"]:h["pw"] + F_ * A].view(F_, A)
        pb = self.flat[h["pb"]:h["pb"] + A]
        vw = self.flat[h["vw"]:h["vw"] + F_].view(F_, 1)
        vb = self.flat[h["vb"]:h["vb"] + 1]
        return pw, pb, vw, vb

    def lstm(self):
        ls = self.layout.lstm
        H = ls["H"]
        k = self.flat[ls["kernel"]:ls["kernel"] + (ls["din"] + H) * 4 * H].view(ls["din"] + H, 4 * H)
        b = self.flat[ls["bias"]:ls["bias"] + 4 * H]
        return k, b

    def tensor(self, name: str) -> torch.Tensor:
        s = self.layout.by_name[name]
        return self.flat[s.offset:s.offset + s.numel].view(s.shape)

    def named_tensors(self) -> Dict[str, torch.Tensor]:
        return {s.name: self.tensor(s.name) for s in self.layout.segments}


# ---------------------------------------------------------------------------
# reference (oracle) forward
# ---------------------------------------------------------------------------
def module_type(spec, j: int) -> int:
    """Supervised module2 kind (pathnet.py:137-168): 0 skip, 1 fc+relu, 2 residual. RL nets: 1."""
    if spec.module_types is None:
        return 1
    return int(spec.module_types[j % len(spec.module_types)])


def bf16_ste(x: torch.Tensor) -> torch.Tensor:
    """Round to bf16 in the forward pass, identity gradient (emulates bf16 storage)."""
    return x + (x.to(torch.bfloat16).float() - x).detach()


def f16_ste(x: torch.Tensor) -> torch.Tensor:
    """Round to fp16 in the forward pass, identity gradient (the HIP uint8-input conv layer's weight copy)."""
    return x + (x.to(torch.float16).float() - x).detach()


def trunk_forward_ref(store: ParamStore, x: torch.Tensor, mask: torch.Tensor,
                      W_override: Optional[List[torch.Tensor]] = None,
                      b_override: Optional[List[torch.Tensor]] = None,
                      emulate_bf16: bool = False) -> torch.Tensor:
    """Dense masked PathNet trunk.

    x    : [B, *input_shape] float (NHWC for pixels, already scaled to [0,1])
    mask : [B, L, M] float (expressed genotype of each sample's path)
    emulate_bf16: round weights and every layer output to bf16 (the HIP
                  kernels' storage precision; fp32 accumulation either way).  A
                  first conv layer (uint8 pixels in the HIP engine) keeps fp16
                  weights there (csrc/conv_fast.hip fp16-offset path), so it is
                  rounded to fp16 instead.
    returns [B, feature_dim]
    """
    cfg = store.cfg
    B = x.shape[0]
    M = cfg.M
    h = x
    for l, spec in enumerate(cfg.layers):
        li = store.layout.layer_info[l]
        W = store.W(l) if W_override is None else W_override[l]
        b = store.b(l) if b_override is None else b_override[l]
        if emulate_bf16:
            W = f16_ste(W) if (l == 0 and spec.kind == "conv") else bf16_ste(W)
        m = mask[:, l, :]
        cout = li["cout"]
        if spec.kind == "conv":
            k = spec.kernel
            cin = li["cin"]
            Wc = W.reshape(M, k, k, cin, cout).permute(0, 4, 3, 1, 2).reshape(M * cout, cin, k, k)
            y = F.conv2d(h.permute(0, 3, 1, 2), Wc, b.reshape(-1), stride=spec.stride)
            Ho, Wo = y.shape[2], y.shape[3]
            y = F.relu(y).view(B, M, cout, Ho, Wo) * m[:, :, None, None, None]
            h = y.sum(1).permute(0, 2, 3, 1)
        else:
            hf = h.reshape(B, -1)
            pre = torch.einsum("bk,mkc->bmc", hf, W) + b[None]
            outs = []
            for j in range(M):
                t = module_type(spec, j)
                if t == 0:
                    o = hf
                elif t == 1:
                    o = F.relu(pre[:, j])
                else:
                    o = F.relu(pre[:, j]) + hf
                outs.append(o * m[:, j:j + 1])
            h = torch.stack(outs, 1).sum(1)
        if emulate_bf16 and l < cfg.L - 1:
            h = bf16_ste(h)
    h = h.reshape(B, -1)
    if cfg.trunk_scale == "M":
        h = h / M
    if emulate_bf16:
        h = bf16_ste(h)
    return h


def lstm_cell_ref(x, h, c, kernel, bias, forget_bias: float = 1.0):
    """TF BasicLSTMCell (gate order i, j, f, o; forget_bias=1.0)."""
    z = torch.cat([x, h], 1) @ kernel + bias
    i, j, f, o = z.chunk(4, 1)
    c2 = c * torch.sigmoid(f + forget_bias) + torch.sigmoid(i) * torch.tanh(j)
    h2 = torch.tanh(c2) * torch.sigmoid(o)
    return h2, c2


def heads_ref(store: ParamStore, feat: torch.Tensor, task: int = 0):
    pw, pb, vw, vb = store.head(task)
    logits = feat @ pw + pb
    value = (feat @ vw + vb).squeeze(-1)
    return logits, value


def count_params(cfg: PathNetConfig) -> int:
    return ParamLayout(cfg).numel


def forward_flops_per_sample(cfg: PathNetConfig, active: Optional[np.ndarray] = None) -> float:
    """MAC*2 per sample for a trunk with ``active[l]`` modules per layer (dense: M)."""
    shapes = cfg.layer_shapes()
    fl = 0.0
    for l, (spec, (ins, outs, K, cin)) in enumerate(zip(cfg.layers, shapes)):
        n = cfg.M if active is None else active[l]
        pos = int(np.prod(outs[:-1])) if spec.kind == "conv" else 1
        fl += 2.0 * pos * K * spec.out * n
    return fl
