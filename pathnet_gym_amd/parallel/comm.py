"""Per-update communication: ONE fused all-reduce over xGMI.

The reference moves every variable through gRPC on every env step (call
sites C1-C12 in SURVEY.md section 2.7).  Here weights are replicated and an
update exchanges exactly one flat fp32 buffer::

    [ active-module gradients | fitness[P_total] | counters ]

* gradients: only modules active in SOME path of the population and not
  frozen, plus the always-trainable heads/LSTM (BASELINE north star:
  "A2C rollout gradients are all-reduced only over active-path
  parameters").  Modules are contiguous chunks of the flat buffer, so the
  pack is a list of ranges; when the union covers most of the network one
  dense range is used instead (cheaper than gather/scatter).
* fitness: each rank writes its own paths' slots, the rest are 0, so the
  SUM is an all-gather (replaces PS polling C5/C6).
* counters: agent steps / episodes (replaces the racy global_step RMW, C4).

Every rank then runs the replicated GA (``algo/ga.py``) on the identical
fitness vector, so genotype broadcasts are unnecessary in the fused mode.
``GatherBroadcastComm`` implements the explicit variant (all-gather of
fitness + RCCL broadcast of the winner genotype table from rank 0), used by
``--ga_sync gather_bcast`` and in tests to check both agree.

Bucket sizing for xGMI: the whole buffer is <= 17 MB, a single ring
all-reduce moves 2*(w-1)/w*S per GPU, ~0.2 ms at 153 GB/s per link, so one
bucket (no splitting) minimises the latency-dominated cost.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np
import torch

from ..models.pathnet import ParamLayout
from .dist import DistContext


def active_ranges(layout: ParamLayout, expressed: np.ndarray, frozen: np.ndarray) -> List[Tuple[int, int]]:
    """Contiguous flat-buffer ranges holding trainable gradients.

    expressed: [P_total, L, M] masks of the WHOLE population.
    """
    union = (np.asarray(expressed) > 0.5).any(0) & ~(np.asarray(frozen) > 0.5)
    ranges = []
    for l in range(layout.cfg.L):
        for j in range(layout.cfg.M):
            if union[l, j]:
                ranges.append(layout.module_range(l, j))
    # heads / lstm: everything after the trunk
    ranges.append((layout.trunk_numel, layout.numel))
    merged = []
    for s, e in sorted(ranges):
        if merged and merged[-1][1] == s:
            merged[-1] = (merged[-1][0], e)
        else:
            merged.append((s, e))
    return merged


class FusedUpdateComm:
    NCOUNTERS = 4   # agent steps, episodes finished, sum of finished returns, spare

    def __init__(self, ctx: DistContext, layout: ParamLayout, P_total: int, P_local: int, device,
                 dense_threshold: float = 0.75):
        self.ctx = ctx
        self.layout = layout
        self.P_total, self.P_local = P_total, P_local
        self.offset = ctx.rank * P_local
        self.device = device
        self.dense_threshold = dense_threshold
        self.ranges = [(0, layout.numel)]
        self.index = None
        self.ngrad = layout.numel
        self.buf = torch.zeros(layout.numel + P_total + self.NCOUNTERS, dtype=torch.float32, device=device)
        # static device copy of the reduced [fitness | counters] (read by the device GA / non-finite skip)
        self.small_dev = torch.zeros(P_total + self.NCOUNTERS, dtype=torch.float32, device=device)
        self.fit_reduced = self.small_dev[:P_total]
        self.cnt_reduced = self.small_dev[P_total:]
        pin = torch.device(device).type == "cuda"
        self.host_small = [torch.zeros(P_total + self.NCOUNTERS, dtype=torch.float32, pin_memory=pin) for _ in range(2)]
        self._flip = 0
        self.force_dense = False
        self.bytes_last = 0

    def plan(self, expressed_all: np.ndarray, frozen: np.ndarray):
        rng = active_ranges(self.layout, expressed_all, frozen)
        n = sum(e - s for s, e in rng)
        if self.force_dense or n >= self.dense_threshold * self.layout.numel:
            self.ranges = [(0, self.layout.numel)]
            self.index = None
            self.ngrad = self.layout.numel
        else:
            self.ranges = rng
            idx = np.concatenate([np.arange(s, e, dtype=np.int64) for s, e in rng])
            self.index = torch.from_numpy(idx).to(self.device)
            self.ngrad = int(n)

    def exchange_async(self, grad: torch.Tensor, fitness_local: torch.Tensor, counters: torch.Tensor, extra=None):
        """Pipelined variant: reduce on the stream, start a non-blocking D2H of [fitness | counters] (+ ``extra``)
        into a pinned double buffer and return a handle for ``collect``; the host does not wait."""
        P = self.P_total
        if not self.ctx.enabled:
            self.small_dev[:P].copy_(fitness_local)
            self.small_dev[P:].copy_(counters)
            self.bytes_last = 0
        else:
            n = self.ngrad
            buf = self.buf
            if self.index is None:
                buf[:n].copy_(grad)
            else:
                buf[:n].copy_(grad.index_select(0, self.index))
            fit = buf[n:n + P]
            fit.zero_()
            fit[self.offset:self.offset + self.P_local].copy_(fitness_local)
            buf[n + P:n + P + self.NCOUNTERS].copy_(counters)
            view = buf[:n + P + self.NCOUNTERS]
            self.ctx.all_reduce_(view)
            self.bytes_last = view.numel() * 4
            if self.index is None:
                grad.copy_(buf[:n])
            else:
                grad.index_copy_(0, self.index, buf[:n])
            self.small_dev.copy_(buf[n:n + P + self.NCOUNTERS])
        hb = self.host_small[self._flip]
        ex = None
        if extra is not None:
            if getattr(self, "_extra_host", None) is None or self._extra_host[0].shape != extra.shape:
                self._extra_host = [torch.zeros(extra.shape, dtype=extra.dtype, pin_memory=hb.is_pinned())
                                    for _ in range(2)]
            ex = self._extra_host[self._flip]
            ex.copy_(extra, non_blocking=True)
        self._flip ^= 1
        hb.copy_(self.small_dev, non_blocking=True)
        ev = torch.cuda.Event() if hb.is_pinned() else None
        if ev is not None:
            ev.record()
        return (ev, hb, ex)

    def collect(self, handle):
        ev, hb, ex = handle
        if ev is not None:
            ev.synchronize()
        h = hb.numpy()
        P = self.P_total
        return h[:P].copy(), h[P:].copy(), (ex.numpy().copy() if ex is not None else None)

    def exchange(self, grad: torch.Tensor, fitness_local: torch.Tensor, counters: torch.Tensor):
        """All-reduce in place. Returns (fitness_all [P_total] cpu numpy, counters_sum cpu numpy)."""
        if not self.ctx.enabled:
            # single rank: nothing to reduce -- read back fitness + counters in ONE small D2H copy
            P = self.P_total
            small = self.buf[:P + self.NCOUNTERS]
            small[:P].copy_(fitness_local)
            small[P:].copy_(counters)
            self.small_dev.copy_(small)
            self.bytes_last = 0
            host = small.cpu().numpy()
            return host[:P].copy(), host[P:].copy()
        n = self.ngrad
        P = self.P_total
        buf = self.buf
        if self.index is None:
            buf[:n].copy_(grad)
        else:
            buf[:n].copy_(grad.index_select(0, self.index))
        fit = buf[n:n + P]
        fit.zero_()
        fit[self.offset:self.offset + self.P_local].copy_(fitness_local)
        buf[n + P:n + P + self.NCOUNTERS].copy_(counters)
        view = buf[:n + P + self.NCOUNTERS]
        self.ctx.all_reduce_(view)
        self.bytes_last = view.numel() * 4
        if self.index is None:
            grad.copy_(buf[:n])
        else:
            grad.index_copy_(0, self.index, buf[:n])
        self.small_dev.copy_(buf[n:n + P + self.NCOUNTERS])
        host = view[n:].cpu().numpy()
        return host[:P].copy(), host[P:].copy()


class GatherBroadcastComm(FusedUpdateComm):
    """Explicit variant: grad all-reduce, fitness all-gather, genotype broadcast."""

    def exchange(self, grad, fitness_local, counters):
        n = self.ngrad
        if self.index is None:
            self.ctx.all_reduce_(grad)
        else:
            g = grad.index_select(0, self.index)
            self.ctx.all_reduce_(g)
            grad.index_copy_(0, self.index, g)
        fit = self.ctx.all_gather(fitness_local.float())
        self.fit_reduced.copy_(fit.reshape(-1))
        c = counters.clone()
        self.ctx.all_reduce_(c)
        self.cnt_reduced.copy_(c)
        self.bytes_last = (n + self.P_total + self.NCOUNTERS) * 4
        return fit.cpu().numpy(), c.cpu().numpy()

    def broadcast_genotypes(self, genotypes: np.ndarray) -> np.ndarray:
        t = torch.from_numpy(np.ascontiguousarray(genotypes.astype(np.uint8))).to(self.device)
        self.ctx.broadcast_(t, 0)
        return t.cpu().numpy().astype(np.float32)
