"""Pipelined HIP updates: a skipped (non-finite) optimizer step is charged to the update it belongs to, and the
last step before ``flush()`` reaches the guard too (runtime/guard.py; trainer._collect / flush)."""
import numpy as np
import pytest
import torch

from pathnet_gym_amd.config import preset

pytestmark = pytest.mark.gpu


def test_pipelined_skip_is_attributed_to_its_update(hip_lib):
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    cfg = preset("pong")
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 4, 16, 2
    cfg.ga.backend = "device"
    cfg.max_nonfinite = 5
    tr = PathNetTrainer(cfg, device="cuda")
    assert tr.pipelined
    eng = tr.engine
    orig = eng.optimizer_step
    poison = {3, 6}

    def step(lr, **kw):
        if tr.updates + 1 in poison:            # the optimizer step of update 3 / 6 sees a NaN gradient
            eng.grad_flat[7] = float("nan")
        orig(lr, **kw)
    eng.optimizer_step = step
    seen = {}
    for _ in range(5):
        st = tr.update()
        if st.skipped:
            seen[st.skipped_update] = tr.updates
    # update 3's optimizer status travels with update 4's report, which update() call 5 collects: it is named as
    # update 3 there
    assert seen == {3: 5}, seen
    st = tr.update()                            # update 6: poisoned, still in flight
    assert not st.skipped
    st = tr.flush()
    assert st.skipped and st.skipped_update == 6
    assert tr.guard.skipped == 2
    assert torch.isfinite(tr.model.store.flat).all()
