"""Failure detection: non-finite gradient guard + hang watchdog.

The reference has no failure handling beyond TF's Supervisor; a dead worker
blocks its coordinator forever (doom_pathnet.py:246-250).
Here every rank runs the same synchronous loop, so failures are handled
collectively:

* ``NonFiniteGuard``: the update's non-finite gradient count travels in the
  spare slot of the fused all-reduce buffer (``parallel/comm.py``), so EVERY
  rank sees the same global count and takes the same decision -- skip the
  optimizer step (weights and RMSProp slots untouched), and raise
  ``NonFiniteError`` after ``max_consecutive`` bad updates.  No extra
  collective, no extra host sync.
* ``Watchdog``: a daemon thread that fires when no update has completed for
  ``timeout_s`` (a hung collective, a wedged kernel, a dead peer): it dumps
  every Python thread's stack and the last traced phase to stderr, then
  (``abort=True``) terminates the process so the launcher (torchrun
  ``--max-restarts``) can restart the job from the last checkpoint
  (``--resume``).  RCCL's own timeout is set at ``init_process_group``.
"""
from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time
from typing import Callable, Optional


class NonFiniteError(RuntimeError):
    pass


class X3RangeError(FloatingPointError):
    """fp32x (split fp16 pairs): a value left the fp16 range.  Bit 0 (value 1) of the status: a weight scaled by
    2^8 -- of any trunk layer (x3_refresh_weights) or the LSTM kernel (lstm_refresh_x3) -- reached 32768 (its pair
    no longer represents it); bit 1 (value 2): an activation written as an fp16 pair (trunk or LSTM state) reached
    65504; bit 2 (value 4, deterministic mode): a weight-gradient contribution left the fixed-point accumulator's range.
    The status travels in the update's all-reduced counters, so every rank raises together.

    Lag: the flags are folded into the counters after each rollout, so an overflow raised by the weight refresh at
    the end of update u surfaces with update u + 1.  ``PathNetTrainer.flush()`` (called at task end and before every
    checkpoint) folds and checks the flags of the last refresh too, so no checkpoint is written over out-of-range
    weights."""

    def __init__(self, status: float, update: int, world: int = 1):
        self.status = status
        bits = int(status) if world == 1 else -1
        what = []
        if bits < 0:
            what.append(f"status sum {status:g} over {world} ranks")
        else:
            if bits & 1:
                what.append("a weight x 2^8 (a trunk layer or the LSTM kernel) left the fp16 range (|W| >= 128)")
            if bits & 2:
                what.append("an activation stored as an fp16 pair reached 65504")
            if bits & 4:
                what.append("deterministic mode: a weight-gradient contribution reached the int64 fixed-point range "
                            "(|g| >= 65536 or NaN, csrc/common.h gacc)")
        super().__init__(f"fp32x range overflow at update {update}: " + "; ".join(what)
                         + " -- use compute_dtype='fp32' for this model / data scale")


class NonFiniteGuard:
    def __init__(self, max_consecutive: int = 3):
        self.max_consecutive = max_consecutive
        self.consecutive = 0
        self.skipped = 0

    def check(self, nonfinite_count: float, update: int) -> bool:
        """True if the optimizer step must be skipped (global decision: the count is all-reduced)."""
        if nonfinite_count > 0:
            self.consecutive += 1
            self.skipped += 1
            if self.consecutive >= self.max_consecutive:
                raise NonFiniteError(f"{int(nonfinite_count)} non-finite gradient entries in "
                                     f"{self.consecutive} consecutive updates (last update {update})")
            return True
        self.consecutive = 0
        return False


class Watchdog:
    def __init__(self, timeout_s: float, abort: bool = True, phase: Optional[Callable[[], str]] = None,
                 stream=None):
        self.timeout_s = timeout_s
        self.abort = abort
        self.phase = phase
        self.stream = stream or sys.stderr
        self.fired = False
        self._last = time.monotonic()
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, name="pathnet-watchdog", daemon=True)
        self._t.start()

    def beat(self):
        self._last = time.monotonic()

    def _run(self):
        period = max(0.05, min(5.0, self.timeout_s / 4))
        while not self._stop.wait(period):
            idle = time.monotonic() - self._last
            if idle > self.timeout_s and not self.fired:
                self.fired = True
                ph = self.phase() if self.phase else "?"
                print(f"[watchdog] no update completed for {idle:.1f}s (phase: {ph}); thread stacks:",
                      file=self.stream, flush=True)
                try:
                    faulthandler.dump_traceback(file=self.stream, all_threads=True)
                except (ValueError, AttributeError, OSError):
                    pass
                if self.abort:
                    os._exit(124)

    def stop(self):
        self._stop.set()
        self._t.join(timeout=1.0)
