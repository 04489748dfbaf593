"""Standalone HIP multi-tensor TF-RMSProp step for ``RMSPropTF(backend='hip')``.

Same kernels as the engine's captured optimizer phase (``csrc/optim.hip``:
per-segment squared norms -> clip_by_norm -> ApplyRMSProp with epsilon
inside the sqrt, frozen segments skipped), for callers that hold a gradient
outside the engine (e.g. the supervised trainer or tests).
"""
from __future__ import annotations

import torch

from . import _lib

_BLK = 8192


def _tables(opt):
    t = getattr(opt, "_hip_tables", None)
    if t is not None:
        return t
    seg_id, beg, end, blk0 = [], [], [], []
    for i, s in enumerate(opt.layout.segments):
        blk0.append(len(seg_id))
        o = s.offset
        while o < s.offset + s.numel:
            e = min(o + _BLK, s.offset + s.numel)
            seg_id.append(i)
            beg.append(o)
            end.append(e)
            o = e
    blk0.append(len(seg_id))
    dev = opt.flat.device
    t = dict(seg=torch.tensor(seg_id, dtype=torch.int32, device=dev),
             beg=torch.tensor(beg, dtype=torch.int64, device=dev),
             end=torch.tensor(end, dtype=torch.int64, device=dev),
             blk0=torch.tensor(blk0, dtype=torch.int32, device=dev),
             partial=torch.zeros(len(seg_id) + 1, dtype=torch.float32, device=dev),
             status=torch.zeros(1, dtype=torch.float32, device=dev),
             lr=torch.zeros(2, dtype=torch.float32, device=dev))
    opt._hip_tables = t
    return t


def rmsprop_step(opt, grad: torch.Tensor, lr: float) -> None:
    _lib.check(grad, torch.float32, numel=opt.flat.numel(), name="grad")
    t = _tables(opt)
    t["lr"][0:1].fill_(float(lr))
    trainable = opt.seg_trainable.to(torch.uint8)
    _lib.call("launch_rmsprop", opt.flat.data_ptr(), grad.data_ptr(), opt.ms.data_ptr(), opt.mom.data_ptr(),
              t["seg"].data_ptr(), t["beg"].data_ptr(), t["end"].data_ptr(), int(t["seg"].numel()),
              t["partial"].data_ptr(), t["blk0"].data_ptr(), trainable.data_ptr(), t["lr"].data_ptr(),
              t["status"].data_ptr(), opt.decay, opt.momentum, opt.epsilon, opt.clip_norm, _lib.stream())
