"""Failure detection, race (replica divergence) detection and tracing -- CPU."""
import json
import time

import numpy as np
import pytest
import torch

from pathnet_gym_amd.algo.trainer import PathNetTrainer
from pathnet_gym_amd.config import preset
from pathnet_gym_amd.runtime.consistency import check_replicas, state_digest
from pathnet_gym_amd.runtime.guard import NonFiniteError, NonFiniteGuard, Watchdog
from pathnet_gym_amd.utils.tracing import PhaseTracer, performance_line


def _trainer(**kw):
    cfg = preset("cartpole-cpu")
    for k, v in kw.items():
        setattr(cfg, k, v)
    return PathNetTrainer(cfg)


def test_nonfinite_guard_policy():
    g = NonFiniteGuard(max_consecutive=2)
    assert not g.check(0, 0)
    assert g.check(5, 1)
    assert not g.check(0, 2)          # streak reset
    assert g.check(1, 3)
    with pytest.raises(NonFiniteError):
        g.check(1, 4)


def test_trainer_skips_nonfinite_updates_then_raises(tmp_path):
    tr = _trainer(max_nonfinite=2, trace_path=str(tmp_path / "trace.json"))
    tr.update()
    s = tr.model.store.layout.by_name["value.weight"]
    with torch.no_grad():
        tr.model.store.flat[s.offset] = float("nan")
    before = tr.model.store.flat.detach().clone()
    st = tr.update()
    assert st.skipped
    after = tr.model.store.flat.detach()
    ok = torch.isfinite(before)
    assert torch.equal(after[ok], before[ok])            # optimizer step skipped
    with pytest.raises(NonFiniteError):
        tr.update()
    summ = tr.tracer.summary()
    assert {"rollout_backward", "allreduce", "ga"} <= set(summ)
    path = tr.tracer.dump()
    d = json.load(open(path))
    assert d["traceEvents"] and d["traceEvents"][0]["ph"] == "X"


def test_watchdog_fires_without_beats():
    import io
    buf = io.StringIO()
    wd = Watchdog(0.2, abort=False, phase=lambda: "allreduce", stream=buf)
    time.sleep(0.7)
    wd.stop()
    assert wd.fired and "allreduce" in buf.getvalue()
    wd2 = Watchdog(0.5, abort=False)
    for _ in range(6):
        time.sleep(0.1)
        wd2.beat()
    wd2.stop()
    assert not wd2.fired


def test_state_digest_detects_any_change():
    tr = _trainer(check_every=1)
    tr.update()                       # check_replicas runs inside (world 1)
    d0 = state_digest(tr)
    assert torch.equal(d0, state_digest(tr))
    with torch.no_grad():
        tr.model.store.flat[123] += 1e-7
    assert not torch.equal(d0, state_digest(tr))
    d1 = state_digest(tr)
    tr.pop.fitness[0] += 1
    assert not torch.equal(d1, state_digest(tr))
    assert check_replicas(tr)["ok"]


def test_performance_line_format():
    assert performance_line(1000, 10.0) == "### Performance : 1000 STEPS in 10 sec. 100 STEPS/sec. 0.36M STEPS/hour"


def test_phase_tracer_gpu_events_only_when_tracing(tmp_path):
    """The per-phase GPU timing events are recorded only when a trace is written (or asked for), and folded every
    RESOLVE_EVERY phases: the pending list stays bounded (it used to grow by 8 live events per update)."""
    from pathnet_gym_amd.utils.tracing import PhaseTracer
    t = PhaseTracer(enabled=True)
    assert not t.cuda
    for _ in range(10):
        with t.phase("x"):
            pass
    assert t.counts["x"] == 10 and not t._pending
    t2 = PhaseTracer(enabled=True, path=str(tmp_path / "tr.json"))
    assert t2.cuda == torch.cuda.is_available()
    for _ in range(3 * PhaseTracer.RESOLVE_EVERY):
        with t2.phase("y"):
            pass
    assert len(t2._pending) < PhaseTracer.RESOLVE_EVERY + 1
