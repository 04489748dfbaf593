"""Phase tracing: per-update GPU/host timing and Chrome-trace export.

The reference's only instrumentation is the "### Performance" line every
1000 local steps on worker 0 (a3c_training_thread.py:236-241).  This tracer
brackets each phase of an update (rollout+backward, all-reduce, optimizer,
GA) with ``torch.cuda.Event`` pairs on the compute stream (GPU time, no
extra sync: events are resolved lazily, one update behind) and host wall
clock, keeps running totals, and writes a Chrome/Perfetto trace
(``chrome://tracing``) when given a path.  Kernel-level detail comes from
``rocprofv3 --kernel-trace --stats`` (``scripts/gpu.sh "kwin TAG"``).
"""
from __future__ import annotations

import json
import os
import time
from collections import defaultdict
from contextlib import contextmanager
from typing import Dict, List, Optional

import torch


class PhaseTracer:
    RESOLVE_EVERY = 256
    def __init__(self, enabled: bool = True, path: Optional[str] = None, rank: int = 0, max_events: int = 200000,
                 gpu_timing: Optional[bool] = None):
        self.enabled = enabled
        self.path = path
        self.rank = rank
        self.max_events = max_events
        # per-phase GPU timing records two timing events into the stream per phase (~8 per update) and keeps them until
        # resolved: only when a trace is written (or asked for), and folded every RESOLVE_EVERY phases so the pending
        # list stays bounded (unbounded, it grew by 8 live events per update in every bench / solve run)
        self.cuda = torch.cuda.is_available() and (bool(path) if gpu_timing is None else bool(gpu_timing))
        self.totals_ms: Dict[str, float] = defaultdict(float)
        self.gpu_ms: Dict[str, float] = defaultdict(float)
        self.counts: Dict[str, int] = defaultdict(int)
        self.events: List[dict] = []
        self._pending = []
        self.current = "idle"
        self._t0 = time.perf_counter()

    @contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        self.current = name
        ev = None
        if self.cuda:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        t = time.perf_counter()
        try:
            yield
        finally:
            dt = time.perf_counter() - t
            if ev is not None:
                ev[1].record()
                self._pending.append((name, ev))
                if len(self._pending) >= self.RESOLVE_EVERY:
                    self.resolve()
            self.totals_ms[name] += dt * 1e3
            self.counts[name] += 1
            if self.path and len(self.events) < self.max_events:
                self.events.append({"name": name, "ph": "X", "pid": self.rank, "tid": 0,
                                    "ts": (t - self._t0) * 1e6, "dur": dt * 1e6})
            self.current = "idle"

    def resolve(self):
        """Fold completed GPU events into gpu_ms (non-blocking for events still in flight)."""
        keep = []
        for name, (a, b) in self._pending:
            if b.query():
                self.gpu_ms[name] += a.elapsed_time(b)
            else:
                keep.append((name, (a, b)))
        self._pending = keep

    def summary(self) -> Dict[str, Dict[str, float]]:
        self.resolve()
        return {k: {"calls": self.counts[k], "host_ms": round(self.totals_ms[k], 3),
                    "gpu_ms": round(self.gpu_ms.get(k, 0.0), 3)} for k in self.counts}

    def dump(self, path: Optional[str] = None) -> Optional[str]:
        path = path or self.path
        if not path:
            return None
        os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
        with open(path, "w") as f:
            json.dump({"traceEvents": self.events, "displayTimeUnit": "ms",
                       "otherData": {"summary": self.summary()}}, f)
        return path


def performance_line(global_t: int, elapsed: float) -> str:
    """The reference's throughput print (a3c_training_thread.py:236-241)."""
    sps = global_t / max(elapsed, 1e-9)
    return "### Performance : {} STEPS in {:.0f} sec. {:.0f} STEPS/sec. {:.2f}M STEPS/hour".format(
        global_t, elapsed, sps, sps * 3600 / 1000000.)
