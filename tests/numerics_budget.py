"""Error budgets derived from measured values.

Each numerics test reports a dict ``{key: relative error}`` (per layer, per segment, per path ...).  The measured
values of the committed MI355X runs live in ``tests/data/numerics_measured.json`` ({test: {key: error}}); a key's
budget is ``HEADROOM`` x its measured error (at least ``HEADROOM`` x 1e-5: a key measured at 0 -- bit-identical
-- still tolerates the atomic-order noise of the bf16 engine).  A key that was never measured falls back to the test's old loose
budget.  ``PATHNET_RECORD_NUMERICS=<file>`` records instead of checking (still against the loose fallback, so a
broken kernel is never recorded): the file keeps the MAX over recording runs, since the bf16 engine's atomic
weight-gradient reductions make repeated runs differ in the last bits.
"""
import json
import os

HEADROOM = 3.0
MEASURED = os.path.join(os.path.dirname(__file__), "data", "numerics_measured.json")


def _load(path):
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        return json.load(f)


def violations(test, errs, fallback, floor=1e-5):
    """[(key, error, budget)] of every key over its budget (the recorded table, else ``fallback``)."""
    table = _load(MEASURED).get(test, {})
    out = []
    for k, v in errs.items():
        ref = table.get(str(k))
        lim = HEADROOM * max(float(ref), floor) if ref is not None else fallback
        if not v < lim:
            out.append((k, v, lim))
    return out


def check(test, errs, fallback, floor=1e-5):
    """Assert every error in ``errs`` is within budget; in record mode, merge them into the record file."""
    rec = os.environ.get("PATHNET_RECORD_NUMERICS")
    if rec:
        bad = [(k, v) for k, v in errs.items() if not v < fallback]
        assert not bad, ("over the fallback budget, not recorded", test, bad)
        d = _load(rec)
        t = d.setdefault(test, {})
        for k, v in errs.items():
            t[str(k)] = max(float(v), float(t.get(str(k), 0.0)))
        os.makedirs(os.path.dirname(rec) or ".", exist_ok=True)
        with open(rec, "w") as f:
            json.dump(d, f, indent=1, sort_keys=True)
        return
    bad = violations(test, errs, fallback, floor)
    assert not bad, (test, bad)
