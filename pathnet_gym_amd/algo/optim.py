"""RMSProp with TensorFlow ``ApplyRMSProp`` semantics over the flat buffer.

Reference ``rmsprop_applier.py``:
* slots: ``rms`` initialised to 1.0 (:37), ``momentum`` zeros (:39);
* per-TENSOR ``clip_by_norm(g, 40)`` (:104): g * clip / max(||g||, clip);
* ms <- rho*ms + (1-rho)*g^2 ; mom <- mu*mom + lr*g/sqrt(ms+eps) ; var <- var - mom
  (epsilon INSIDE the sqrt, :82-89);
* frozen modules get no apply op at all (a3c_training_thread.py:190-216);
  non-frozen tensors are applied even with zero gradient (rms decays).

Here a "tensor" is a Segment of the flat buffer.  The torch path is the
oracle; the HIP path is two launches (``segment_sqnorm`` + fused
clip/apply that also refreshes the bf16 compute copy).
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from ..models.pathnet import ParamLayout


class RMSPropTF:
    def __init__(self, layout: ParamLayout, flat: torch.Tensor, decay=0.99, momentum=0.0,
                 epsilon=0.1, clip_norm=40.0, backend: str = "torch"):
        self.layout = layout
        self.flat = flat
        self.decay, self.momentum, self.epsilon, self.clip_norm = decay, momentum, epsilon, clip_norm
        self.backend = backend
        dev = flat.device
        self.ms = torch.ones_like(flat)
        self.mom = torch.zeros_like(flat)
        segs = layout.segments
        self.nseg = len(segs)
        self.seg_off = torch.tensor([s.offset for s in segs] + [layout.numel], dtype=torch.int64, device=dev)
        seg_id = np.zeros(layout.numel, np.int64)
        for i, s in enumerate(segs):
            seg_id[s.offset:s.offset + s.numel] = i
        self.seg_id = torch.from_numpy(seg_id).to(dev)
        self.seg_trainable = torch.ones(self.nseg, dtype=torch.bool, device=dev)
        self.last_norms: Optional[torch.Tensor] = None

    def set_frozen(self, frozen_mask: np.ndarray, frozen_tasks=()):
        """frozen_mask [L, M]: exclude every segment of frozen modules (and per-task heads of finished tasks)."""
        tr = np.ones(self.nseg, bool)
        for i, s in enumerate(self.layout.segments):
            if s.layer >= 0 and frozen_mask[s.layer, s.module] > 0.5:
                tr[i] = False
            if s.task >= 0 and s.task in frozen_tasks:
                tr[i] = False
        self.seg_trainable.copy_(torch.from_numpy(tr))

    def segment_norms(self, grad: torch.Tensor) -> torch.Tensor:
        sq = torch.zeros(self.nseg, dtype=torch.float32, device=grad.device)
        sq.index_add_(0, self.seg_id, grad.float() * grad.float())
        return sq.sqrt()

    def step(self, grad: torch.Tensor, lr) -> None:
        if self.backend == "hip":
            from ..ops import optim as hop
            hop.rmsprop_step(self, grad, lr)
            return
        norms = self.segment_norms(grad)
        self.last_norms = norms
        scale = self.clip_norm / torch.maximum(norms, torch.full_like(norms, self.clip_norm))
        g = grad * scale[self.seg_id]
        tr = self.seg_trainable[self.seg_id]
        ms_new = self.decay * self.ms + (1.0 - self.decay) * g * g
        mom_new = self.momentum * self.mom + lr * g / torch.sqrt(ms_new + self.epsilon)
        self.ms = torch.where(tr, ms_new, self.ms)
        self.mom = torch.where(tr, mom_new, self.mom)
        with torch.no_grad():
            self.flat.sub_(torch.where(tr, mom_new, torch.zeros_like(mom_new)))

    def state_dict(self):
        return {"ms": self.ms, "mom": self.mom, "seg_trainable": self.seg_trainable}

    def load_state_dict(self, d):
        self.ms.copy_(d["ms"])
        self.mom.copy_(d["mom"])
        self.seg_trainable.copy_(d["seg_trainable"])


def anneal_lr(lr0: float, global_t: int, max_t: int, task_start: int = 0, mode: str = "per_task") -> float:
    """lr0*(T_max - t)/T_max clamped >= 0 (a3c_training_thread.py:83-87).

    mode "global" reproduces the reference quirk (task 2 runs at t > T_max so
    lr == 0); "per_task" anneals within each task; "none" keeps lr0.
    """
    if mode == "none":
        return lr0
    t = global_t - task_start if mode == "per_task" else global_t
    lr = lr0 * (max_t - t) / max_t
    return max(lr, 0.0)
