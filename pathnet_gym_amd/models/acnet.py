"""Actor-critic PathNet (reference ``GameACPathNetNetwork`` / ``...LSTMNetwork``).

One super-network shared by the whole population; each sample belongs to
one path (batch layout is PATH-MAJOR: sample b of a batch with S samples per
path belongs to path b // S).  The path's expressed genotype selects the
active modules of every layer.

Backends
--------
``torch``  dense masked reference graph (``models/pathnet.py``), used as the
           numerical oracle and on CPU.
``hip``    hand-written CDNA4 kernels (``ops/pathnet_ops.py``): only ACTIVE
           modules are computed (indexed grouped GEMM over the compacted
           per-path module lists), the module sum is fused into the epilogue,
           the uint8 frame stack is consumed directly (1/255 folded into the
           epilogue), ReLU masks are kept as bits for the backward pass.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

from ..algo.ga import compact_active
from ..config import PathNetConfig
from .pathnet import ParamStore, heads_ref, lstm_cell_ref, trunk_forward_ref


class ACPathNet:
    def __init__(self, cfg: PathNetConfig, num_paths: int, device="cpu", backend: str = "torch",
                 seed: int = 1, compute_dtype: Optional[str] = None, deterministic: bool = False):
        self.cfg = cfg
        self.P = num_paths
        self.device = torch.device(device)
        self.backend = backend
        # HIP backend: "bf16" (default) or "fp32" operands; the torch backend always computes in fp32
        self.compute_dtype = compute_dtype or ("bf16" if backend == "hip" else "fp32")
        self.deterministic = deterministic
        self.store = ParamStore(cfg, self.device, seed)
        self.store.flat.requires_grad_(True)
        self.task = 0
        L, M = cfg.L, cfg.M
        self.mask = torch.zeros(num_paths, L, M, device=self.device)
        self.act_idx = torch.full((num_paths, L, M), -1, dtype=torch.int32, device=self.device)
        self.act_cnt = torch.zeros(num_paths, L, dtype=torch.int32, device=self.device)
        self.frozen = np.zeros((L, M), np.float32)
        self.hip = None
        if backend == "hip":
            from ..ops.pathnet_ops import HipPathNet
            self.hip = HipPathNet(self)
            self.hip.set_paths(self.mask.cpu().numpy())

    # ------------------------------------------------------------------
    def set_paths(self, expressed: np.ndarray):
        """Install expressed masks [P, L, M] (in-place: hipGraph-safe addresses)."""
        expressed = np.asarray(expressed, np.float32)
        assert expressed.shape == (self.P, self.cfg.L, self.cfg.M), expressed.shape
        idx, cnt = compact_active(expressed)
        self.mask.copy_(torch.from_numpy(expressed))
        self.act_idx.copy_(torch.from_numpy(idx))
        self.act_cnt.copy_(torch.from_numpy(cnt))
        if self.hip is not None:
            self.hip.set_paths(expressed)

    def set_frozen(self, frozen: np.ndarray):
        self.frozen = np.asarray(frozen, np.float32).copy()
        if self.hip is not None:
            self.hip.set_frozen(self.frozen)

    def init_state(self, batch: int):
        if not self.cfg.use_lstm:
            return None
        H = self.cfg.lstm_size
        z = torch.zeros(batch, H, device=self.device)
        return (z, z.clone())

    # ------------------------------------------------------------------
    def trunk(self, obs: torch.Tensor, samples_per_path: int) -> torch.Tensor:
        B = obs.shape[0]
        assert B == self.P * samples_per_path, (B, self.P, samples_per_path)
        if self.backend == "hip":
            return self.hip.trunk(obs, samples_per_path)
        x = obs.float() * (1.0 / 255.0) if obs.dtype == torch.uint8 else obs.float()
        mask = self.mask.repeat_interleave(samples_per_path, 0)
        return trunk_forward_ref(self.store, x, mask)

    def forward(self, obs: torch.Tensor, samples_per_path: int, state=None):
        """-> logits [B, A], value [B], new_state"""
        feat = self.trunk(obs, samples_per_path)
        if self.cfg.use_lstm:
            k, b = self.store.lstm()
            h, c = state
            h, c = lstm_cell_ref(feat, h, c, k, b)
            feat = h
            state = (h, c)
        if self.backend == "hip":
            logits, value = self.hip.heads(feat, self.task)
        else:
            logits, value = heads_ref(self.store, feat, self.task)
        return logits, value, state

    def parameters_flat(self) -> torch.Tensor:
        return self.store.flat
