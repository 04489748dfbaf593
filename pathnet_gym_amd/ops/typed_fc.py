"""HIP typed-module FC trunk (``csrc/typed_fc.hip``).

This is the forward and backward of an all-FC PathNet trunk whose modules have a type from
``LayerSpec.module_types``: 0 skip, 1 fc+ReLU, 2 residual. These are the supervised builders'
module variants (reference ``pathnet.py:122-196``); the numerics oracle is
``models.pathnet.trunk_forward_ref``. Rows are grouped by path: ``mask`` is
[P, L, M] and row r belongs to path ``r // rows_per_path``. The gradient lands in a flat
buffer shaped like the parameter store, so optimizers see the usual flat layout.
"""
from __future__ import annotations

from typing import List

import torch

from . import _lib


def _types(store) -> List[torch.Tensor]:
    cache = getattr(store, "_typed_fc_types", None)
    if cache is None:
        from ..models.pathnet import module_type
        cfg = store.cfg
        cache = []
        for l, spec in enumerate(cfg.layers):
            if spec.kind != "fc":
                raise NotImplementedError("typed FC trunk: every layer must be fc")
            li = store.layout.layer_info[l]
            t = [module_type(spec, j) for j in range(cfg.M)]
            if any(v != 1 for v in t) and li["K"] != li["cout"]:
                raise ValueError(f"layer {l}: skip/residual modules need in width == out width")
            if li["cout"] > 64 or cfg.M > 16:
                raise NotImplementedError("typed FC trunk: width <= 64 and M <= 16")
            cache.append(torch.tensor(t, dtype=torch.int32, device=store.flat.device))
        store._typed_fc_types = cache
    return cache


class _TypedTrunk(torch.autograd.Function):
    @staticmethod
    def forward(ctx, flat, x, mask, store, rpp):
        cfg = store.cfg
        P = mask.shape[0]
        types = _types(store)
        h = x.contiguous()
        saved_x, saved_relu, masks = [], [], []
        s = _lib.stream()
        for l in range(cfg.L):
            li = store.layout.layer_info[l]
            K, C = li["K"], li["cout"]
            _lib.check(h, torch.float32, shape=(P * rpp, K), name=f"x[{l}]")
            ml = mask[:, l, :].contiguous()
            out = torch.empty(P * rpp, C, dtype=torch.float32, device=x.device)
            relu = torch.empty(P * rpp, cfg.M, C, dtype=torch.uint8, device=x.device)
            _lib.call("launch_typed_fc_fwd", h.data_ptr(), K, flat.data_ptr(), li["offset"], li["chunk"], C, cfg.M,
                      ml.data_ptr(), types[l].data_ptr(), P, rpp, out.data_ptr(), relu.data_ptr(), s)
            saved_x.append(h)
            saved_relu.append(relu)
            masks.append(ml)
            h = out
        ctx.store, ctx.rpp, ctx.P = store, rpp, P
        ctx.saved = (saved_x, saved_relu, masks)
        ctx.save_for_backward(flat)
        return h

    @staticmethod
    def backward(ctx, gout):
        (flat,) = ctx.saved_tensors
        store, rpp, P = ctx.store, ctx.rpp, ctx.P
        saved_x, saved_relu, masks = ctx.saved
        cfg = store.cfg
        types = _types(store)
        gflat = torch.zeros_like(flat)
        g = gout.contiguous().float()
        s = _lib.stream()
        for l in reversed(range(cfg.L)):
            li = store.layout.layer_info[l]
            K, C = li["K"], li["cout"]
            _lib.call("launch_typed_fc_wgrad", saved_x[l].data_ptr(), g.data_ptr(), K, li["offset"], li["chunk"], C,
                      cfg.M, P, masks[l].data_ptr(), types[l].data_ptr(), rpp, saved_relu[l].data_ptr(),
                      gflat.data_ptr(), s)
            if l > 0:
                dx = torch.empty(P * rpp, K, dtype=torch.float32, device=g.device)
                _lib.call("launch_typed_fc_dgrad", g.data_ptr(), K, flat.data_ptr(), li["offset"], li["chunk"], C,
                          cfg.M, masks[l].data_ptr(), types[l].data_ptr(), P, rpp, saved_relu[l].data_ptr(),
                          dx.data_ptr(), s)
                g = dx
        return gflat, None, None, None, None


def typed_trunk_forward(store, x: torch.Tensor, mask_paths: torch.Tensor, rows_per_path: int) -> torch.Tensor:
    """x [P*rows_per_path, K0] fp32, mask_paths [P, L, M] -> features [P*rows_per_path, C_last].

    Differentiable w.r.t. ``store.flat`` (the gradient of x is not formed)."""
    if store.cfg.trunk_scale == "M":
        raise NotImplementedError("typed FC trunk implements trunk_scale='none'")
    P = mask_paths.shape[0]
    if x.shape[0] != P * rows_per_path:
        raise ValueError("x rows must equal P * rows_per_path")
    return _TypedTrunk.apply(store.flat, x.float(), mask_paths.float().contiguous(), store, rows_per_path)
