"""Per-update communication: ONE fused all-reduce over xGMI.

The reference moves every variable through gRPC on every env step (call
sites C1-C12 in SURVEY.md section 2.7).  Here weights are replicated and an
update exchanges exactly one flat fp32 buffer::

    [ active-module gradients | fitness[P_total] | counters ]

* gradients: only modules active in SOME path of the population and not
  frozen, plus the always-trainable heads/LSTM (BASELINE north star:
  "A2C rollout gradients are all-reduced only over active-path
  parameters").  Modules are contiguous chunks of the flat buffer, so the
  pack is a list of ranges (gathered/scattered by ``csrc/comm.hip`` on the
  GPU); only when the union covers >= 95 % of the network is the dense
  buffer reduced instead.  With the device GA the union comes from the GPU
  (``HipEngine.active_union``) so the plan always matches the running rollout.
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
bucket minimises the latency-dominated cost -- except that it would wait for
the LAST backward kernel.  With ``enable_overlap(split_off)`` (HIP engine,
pipelined, world > 1) the update is split at the first layer: bucket 1 =
[gradients at offsets >= split_off (layers 1..L-1 + heads) | fitness |
counters] is all-reduced asynchronously (RCCL runs it on its own stream)
while the first layer's weight-gradient kernel -- the longest backward
kernel, 1.5-2.4 ms at the bench shape -- runs on the compute stream; bucket 2
(the first layer's active modules) follows.  Per element the sums are the
same two-way additions as the single bucket, so at two ranks the result is
bit-identical (tests/test_dist_hip.py).
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np
import torch

from ..models.pathnet import ParamLayout
from .dist import DistContext


def active_union(expressed: np.ndarray, frozen: np.ndarray) -> np.ndarray:
    """[L, M] bool: modules some path of the WHOLE population expresses and that are not frozen."""
    return (np.asarray(expressed) > 0.5).any(0) & ~(np.asarray(frozen) > 0.5)


def union_ranges(layout: ParamLayout, union: np.ndarray) -> List[Tuple[int, int]]:
    """Contiguous flat-buffer ranges holding trainable gradients for a module union (+ the heads/LSTM tail)."""
    union = np.asarray(union).reshape(layout.cfg.L, layout.cfg.M)
    ranges = [layout.module_range(l, j) for l in range(layout.cfg.L) for j in range(layout.cfg.M) if union[l, j]]
    ranges.append((layout.trunk_numel, layout.numel))
    merged = []
    for s, e in sorted(ranges):
        if merged and merged[-1][1] == s:
            merged[-1] = (merged[-1][0], e)
        else:
            merged.append((s, e))
    return merged


def active_ranges(layout: ParamLayout, expressed: np.ndarray, frozen: np.ndarray) -> List[Tuple[int, int]]:
    """Contiguous flat-buffer ranges holding trainable gradients. expressed: [P_total, L, M] of the population."""
    return union_ranges(layout, active_union(expressed, frozen))


class FusedUpdateComm:
    NCOUNTERS = 4   # agent steps, episodes finished, sum of finished returns, spare
    NEXTRA = 8      # report values packed behind them on the single-rank path (exchange_async)

    def __init__(self, ctx: DistContext, layout: ParamLayout, P_total: int, P_local: int, device,
                 dense_threshold: float = 0.95):
        self.ctx = ctx
        self.layout = layout
        self.P_total, self.P_local = P_total, P_local
        self.offset = ctx.rank * P_local
        self.device = torch.device(device)
        self.dense_threshold = dense_threshold
        self.ranges = [(0, layout.numel)]
        self.index = None
        self.ngrad = layout.numel
        self.buf = torch.zeros(layout.numel + P_total + self.NCOUNTERS, dtype=torch.float32, device=device)
        # static device copy of the reduced [fitness | counters] (read by the device GA / non-finite skip), followed
        # by room for the caller's small report: on one rank, exchange_async packs all three with ONE cat and reads
        # them back with ONE D2H copy
        self._small_pack = torch.zeros(P_total + self.NCOUNTERS + self.NEXTRA, dtype=torch.float32, device=device)
        self.small_dev = self._small_pack[:P_total + self.NCOUNTERS]
        self.fit_reduced = self.small_dev[:P_total]
        self.cnt_reduced = self.small_dev[P_total:]
        pin = self.device.type == "cuda"
        self.host_small = [torch.zeros(P_total + self.NCOUNTERS + self.NEXTRA, dtype=torch.float32, pin_memory=pin)
                           for _ in range(2)]
        self._flip = 0
        self.force_dense = False
        self.bytes_last = 0
        # GPU packing: a (src_off, len, dst_off) int64 range table per plan, staged through a pinned double
        # buffer (a plan changes only when the population's module union does)
        cap = layout.cfg.L * layout.cfg.M + 1
        self._gpu_pack = pin
        if pin:
            self._rtab_host = [torch.zeros(cap, 3, dtype=torch.int64, pin_memory=True) for _ in range(2)]
            self._rtab_dev = [torch.zeros(cap, 3, dtype=torch.int64, device=device) for _ in range(2)]
            self._rtab_ev = [None, None]
            self._rtab_flip = 0
        self.rtab = None            # device range table of the current sparse plan (None: dense)
        self.nranges = 0
        self._union_key = None
        self.plans = 0              # number of distinct plans built (diagnostics)
        # split (overlapped) exchange: bucket tables for offsets >= split_off / < split_off
        self.split_off = None
        self.n1 = self.n2 = 0
        self.tab1 = self.tab2 = None
        self.nr1 = self.nr2 = 0
        self.overlap_log = None     # list of per-update timing records when tracing (utils/tracing.py)

    def enable_overlap(self, split_off: int):
        """Split every exchange at flat offset ``split_off`` (the first layer's end) into two async buckets."""
        if not self._gpu_pack:
            raise RuntimeError("the overlapped exchange packs on the GPU (HIP engine)")
        self.split_off = int(split_off)
        self._split_tabs = [[torch.zeros(self.layout.cfg.L * self.layout.cfg.M + 1, 3, dtype=torch.int64,
                                         device=self.device) for _ in range(2)] for _ in range(2)]
        self._split_host = [[torch.zeros(self.layout.cfg.L * self.layout.cfg.M + 1, 3, dtype=torch.int64,
                                          pin_memory=True) for _ in range(2)] for _ in range(2)]
        self._split_ev = [None, None]
        self._split_flip = 0
        self._union_key = None
        self._plan_split([(0, self.layout.numel)])      # dense until the first module union arrives

    # -- planning ---------------------------------------------------------------
    def plan(self, expressed_all: np.ndarray, frozen: np.ndarray):
        """Host view: plan from the population's expressed masks [P_total, L, M] and the frozen mask."""
        self.plan_union(active_union(expressed_all, frozen))

    def plan_union(self, union: np.ndarray):
        """Plan from an [L, M] module union (e.g. read back from the device GA, runtime/engine.py)."""
        union = np.asarray(union).astype(bool).reshape(self.layout.cfg.L, self.layout.cfg.M)
        key = (union.tobytes(), self.force_dense)
        if key == self._union_key:
            return
        self._union_key = key
        self.plans += 1
        rng = union_ranges(self.layout, union)
        n = sum(e - s for s, e in rng)
        if self.split_off is not None:
            self._plan_split(rng if not self.force_dense else [(0, self.layout.numel)])
            return
        if self.force_dense or n >= self.dense_threshold * self.layout.numel:
            self.ranges = [(0, self.layout.numel)]
            self.index = None
            self.rtab = None
            self.ngrad = self.layout.numel
            return
        self.ranges = rng
        self.ngrad = int(n)
        if self._gpu_pack:
            f = self._rtab_flip
            self._rtab_flip ^= 1
            if self._rtab_ev[f] is not None:
                self._rtab_ev[f].synchronize()          # the previous upload from this pinned buffer finished
            tab = np.zeros((len(rng), 3), np.int64)
            d = 0
            for i, (s, e) in enumerate(rng):
                tab[i] = (s, e - s, d)
                d += e - s
            self._rtab_host[f][:len(rng)].copy_(torch.from_numpy(tab))
            self._rtab_dev[f].copy_(self._rtab_host[f], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._rtab_ev[f] = ev
            self.rtab = self._rtab_dev[f]
            self.nranges = len(rng)
            self.index = None
        else:
            idx = np.concatenate([np.arange(s, e, dtype=np.int64) for s, e in rng])
            self.index = torch.from_numpy(idx).to(self.device)

    def _plan_split(self, rng):
        so = self.split_off
        r1 = [(max(s, so), e) for s, e in rng if e > so]
        r2 = [(s, min(e, so)) for s, e in rng if s < so]
        self.ranges = rng
        self.n1 = sum(e - s for s, e in r1)
        self.n2 = sum(e - s for s, e in r2)
        self.ngrad = self.n1 + self.n2
        f = self._split_flip
        self._split_flip ^= 1
        if self._split_ev[f] is not None:
            self._split_ev[f].synchronize()
        for b, rr in enumerate((r1, r2)):
            tab = np.zeros((max(1, len(rr)), 3), np.int64)
            d = 0
            for i, (s, e) in enumerate(rr):
                tab[i] = (s, e - s, d)
                d += e - s
            self._split_host[f][b][:len(tab)].copy_(torch.from_numpy(tab))
            self._split_tabs[f][b].copy_(self._split_host[f][b], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._split_ev[f] = ev
        self.tab1, self.tab2 = self._split_tabs[f]
        self.nr1, self.nr2 = len(r1), len(r2)

    def _pack_tab(self, grad, packed_off: int, tab, nr: int, n: int, unpack: int):
        if n == 0 or nr == 0:
            return
        from ..ops import _lib
        _lib.call("launch_pack_ranges", grad.data_ptr(), self.buf.data_ptr() + packed_off * 4, tab.data_ptr(), nr, n,
                  unpack, _lib.stream())

    def exchange_async_split(self, grad: torch.Tensor, fitness_local: torch.Tensor, counters: torch.Tensor,
                             run_tail, extra=None):
        """Overlapped form of ``exchange_async``: bucket 1 (offsets >= split_off, fitness, counters) goes out
        asynchronously, then ``run_tail()`` enqueues the first layer's backward on the compute stream (it runs while
        bucket 1 is reduced), then bucket 2 (offsets < split_off).  Both are waited for before unpacking."""
        import time
        import torch.distributed as dist
        P = self.P_total
        n1, n2 = self.n1, self.n2
        m = n1 + P + self.NCOUNTERS
        buf = self.buf
        rec = {} if self.overlap_log is not None else None
        self._pack_tab(grad, 0, self.tab1, self.nr1, n1, 0)
        fit = buf[n1:n1 + P]
        fit.zero_()
        fit[self.offset:self.offset + self.P_local].copy_(fitness_local)
        buf[n1 + P:m].copy_(counters)
        if rec is not None:
            rec["b1_issue"] = time.perf_counter()
        w1 = dist.all_reduce(buf[:m], op=dist.ReduceOp.SUM, async_op=True)
        if rec is not None:
            fut = w1.get_future()
            fut.then(lambda _f: rec.__setitem__("b1_done", time.perf_counter()))
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            rec["tail_enqueue"] = time.perf_counter()
        run_tail()
        if rec is not None:
            e1.record()
        self._pack_tab(grad, m, self.tab2, self.nr2, n2, 0)
        w2 = dist.all_reduce(buf[m:m + n2], op=dist.ReduceOp.SUM, async_op=True) if n2 > 0 else None
        w1.wait()
        self._pack_tab(grad, 0, self.tab1, self.nr1, n1, 1)
        self.small_dev.copy_(buf[n1:m])
        if w2 is not None:
            w2.wait()
            self._pack_tab(grad, m, self.tab2, self.nr2, n2, 1)
        self.bytes_last = (m + n2) * 4
        if rec is not None:
            e1.synchronize()
            rec["b_all_done"] = time.perf_counter()
            rec["tail_gpu_ms"] = e0.elapsed_time(e1)
            rec["n1"], rec["n2"] = n1, n2
            self.overlap_log.append(rec)
        return self._readback(extra)

    def _readback(self, extra):
        """Start the D2H of the reduced [fitness | counters] (+ ``extra``) into the pinned double buffer."""
        hb = self.host_small[self._flip]
        ex = None
        if isinstance(extra, (list, tuple)):
            extra = torch.cat([e.reshape(-1) for e in extra])
        if extra is not None:
            if getattr(self, "_extra_host", None) is None or self._extra_host[0].shape != extra.shape:
                self._extra_host = [torch.zeros(extra.shape, dtype=extra.dtype, pin_memory=hb.is_pinned())
                                    for _ in range(2)]
            ex = self._extra_host[self._flip]
            ex.copy_(extra, non_blocking=True)
        self._flip ^= 1
        hb[:self.small_dev.numel()].copy_(self.small_dev, non_blocking=True)
        ev = torch.cuda.Event() if hb.is_pinned() else None
        if ev is not None:
            ev.record()
        return (ev, hb, ex)

    @property
    def dense(self) -> bool:
        return self.index is None and self.rtab is None

    def _pack(self, grad: torch.Tensor, n: int):
        if self.dense:
            self.buf[:n].copy_(grad)
        elif self.rtab is not None:
            from ..ops import _lib
            _lib.call("launch_pack_ranges", grad.data_ptr(), self.buf.data_ptr(), self.rtab.data_ptr(), self.nranges,
                      n, 0, _lib.stream())
        else:
            self.buf[:n].copy_(grad.index_select(0, self.index))

    def _unpack(self, grad: torch.Tensor, n: int):
        if self.dense:
            grad.copy_(self.buf[:n])
        elif self.rtab is not None:
            from ..ops import _lib
            _lib.call("launch_pack_ranges", grad.data_ptr(), self.buf.data_ptr(), self.rtab.data_ptr(), self.nranges,
                      n, 1, _lib.stream())
        else:
            grad.index_copy_(0, self.index, self.buf[:n])

    def _reduce(self, grad: torch.Tensor, fitness_local: torch.Tensor, counters: torch.Tensor) -> int:
        """Pack [active grads | fitness (own slots) | counters], ONE all-reduce, unpack. Returns n."""
        n = self.ngrad
        P = self.P_total
        buf = self.buf
        self._pack(grad, n)
        fit = buf[n:n + P]
        fit.zero_()
        fit[self.offset:self.offset + self.P_local].copy_(fitness_local)
        buf[n + P:n + P + self.NCOUNTERS].copy_(counters)
        view = buf[:n + P + self.NCOUNTERS]
        self.ctx.all_reduce_(view)
        self.bytes_last = view.numel() * 4
        self._unpack(grad, n)
        self.small_dev.copy_(buf[n:n + P + self.NCOUNTERS])
        return n

    # -- exchange ---------------------------------------------------------------
    def exchange_async(self, grad: torch.Tensor, fitness_local: torch.Tensor, counters: torch.Tensor, extra=None):
        """Pipelined variant: reduce on the stream, start a non-blocking D2H of [fitness | counters] (+ ``extra``)
        into a pinned double buffer and return a handle for ``collect``; the host does not wait."""
        P, NC = self.P_total, self.NCOUNTERS
        if not self.ctx.enabled:
            self.bytes_last = 0
            parts = [fitness_local.reshape(-1), counters.reshape(-1)]
            if isinstance(extra, (list, tuple)):
                parts += [e.reshape(-1) for e in extra]
            ne = sum(int(t.numel()) for t in parts) - P - NC
            if (extra is None or isinstance(extra, (list, tuple))) and ne <= self.NEXTRA and \
                    all(t.dtype == torch.float32 for t in parts):
                # one cat into [fitness | counters | report] and one D2H (instead of 2 + 2 copies and 2 D2H)
                n = P + NC + ne
                torch.cat(parts, out=self._small_pack[:n])
                hb = self.host_small[self._flip]
                self._flip ^= 1
                hb[:n].copy_(self._small_pack[:n], non_blocking=True)
                ev = torch.cuda.Event() if hb.is_pinned() else None
                if ev is not None:
                    ev.record()
                return (ev, hb, ne)
            self.small_dev[:P].copy_(fitness_local)
            self.small_dev[P:].copy_(counters)
        else:
            self._reduce(grad, fitness_local, counters)
        return self._readback(extra)

    def collect(self, handle):
        """(fitness [P_total], counters [NCOUNTERS], extra or None) of an ``exchange_async*`` handle; waits for its
        D2H.  ``extra``: the report packed behind the counters (an int count in the handle) or its own buffer."""
        ev, hb, ex = handle
        if ev is not None:
            ev.synchronize()
        h = hb.numpy()
        P, NC = self.P_total, self.NCOUNTERS
        if isinstance(ex, int):
            extra = h[P + NC:P + NC + ex].copy() if ex > 0 else None
        else:
            extra = ex.numpy().copy() if ex is not None else None
        return h[:P].copy(), h[P:P + NC].copy(), extra

    def exchange(self, grad: torch.Tensor, fitness_local: torch.Tensor, counters: torch.Tensor):
        """All-reduce in place. Returns (fitness_all [P_total] cpu numpy, counters_sum cpu numpy)."""
        P = self.P_total
        if not self.ctx.enabled:
            # single rank: nothing to reduce -- read back fitness + counters in ONE small D2H copy
            small = self.buf[:P + self.NCOUNTERS]
            small[:P].copy_(fitness_local)
            small[P:].copy_(counters)
            self.small_dev.copy_(small)
            self.bytes_last = 0
            host = small.cpu().numpy()
            return host[:P].copy(), host[P:].copy()
        n = self._reduce(grad, fitness_local, counters)
        host = self.buf[n:n + P + self.NCOUNTERS].cpu().numpy()
        return host[:P].copy(), host[P:].copy()


class GatherBroadcastComm(FusedUpdateComm):
    """Explicit variant: grad all-reduce, fitness all-gather, genotype broadcast."""

    def exchange(self, grad, fitness_local, counters):
        n = self.ngrad
        if self.dense:
            self.ctx.all_reduce_(grad)
        else:
            self._pack(grad, n)
            self.ctx.all_reduce_(self.buf[:n])
            self._unpack(grad, n)
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
