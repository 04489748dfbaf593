"""Metrics: JSONL event log + throughput meter (+ optional TensorBoard).

Reference observability: a "### Performance" print
every 1000 local steps (``a3c_training_thread.py:236-241``), the
coordinator's "<step> Step Score: <s>" per tournament
(``doom_pathnet.py:256``) and a TensorBoard ``score`` scalar.  Here every
event is one JSON line (machine readable); the same lines are echoed in the
reference's human format.  The throughput meter fixes the reference's
task-2 timer artefact by measuring delta-steps / delta-time.
"""
from __future__ import annotations

import json
import os
import sys
import time
from typing import Optional


class MetricsLogger:
    def __init__(self, path: Optional[str] = None, echo: bool = True, tensorboard_dir: Optional[str] = None):
        self.path = path
        self.echo = echo
        self.fh = None
        if path:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            self.fh = open(path, "a")
        self.tb = None
        if tensorboard_dir:
            try:
                from torch.utils.tensorboard import SummaryWriter   # needs the tensorboard package
                self.tb = SummaryWriter(tensorboard_dir)
            except Exception:
                self.tb = None
        self._last_t = time.time()
        self._last_step = 0

    def log(self, kind: str, **kw):
        rec = {"t": round(time.time(), 3), "kind": kind, **kw}
        line = json.dumps(rec, default=_jsonable)
        if self.fh:
            self.fh.write(line + "\n")
            self.fh.flush()
        if self.echo:
            if kind == "tournament":
                print(f"{kw.get('step')} Step Score: {kw.get('score')}")
            elif kind == "perf":
                sps = kw.get("steps_per_sec", 0.0)
                print(f"### Performance : {kw.get('step')} STEPS. {sps:.0f} STEPS/sec. "
                      f"{sps * 3600 / 1e6:.2f}M STEPS/hour")
            else:
                print(line)
            sys.stdout.flush()
        if self.tb is not None and kind in ("tournament", "perf"):
            step = kw.get("step", 0)
            for k, v in kw.items():
                if isinstance(v, (int, float)) and k != "step":
                    self.tb.add_scalar(f"{kind}/{k}", v, step)

    def rate(self, step: int) -> float:
        """delta-steps / delta-time since the previous call."""
        now = time.time()
        r = (step - self._last_step) / max(now - self._last_t, 1e-9)
        self._last_t, self._last_step = now, step
        return r

    def close(self):
        if self.fh:
            self.fh.close()
        if self.tb is not None:
            self.tb.close()


def _jsonable(o):
    try:
        import numpy as np
        if isinstance(o, np.ndarray):
            return o.tolist()
        if isinstance(o, (np.integer,)):
            return int(o)
        if isinstance(o, (np.floating,)):
            return float(o)
    except Exception:
        pass
    return str(o)
