"""HIP typed-module PathNet trunk for the supervised builders (``csrc/typed_fc.hip``).

Module kinds (reference ``pathnet.py:122-196``):

* fc layers: per-module type from ``LayerSpec.module_types`` -- 0 skip, 1 fc + ReLU (``module``), 2 residual
  (``module2``);
* conv layers (``conv_module``, ``pathnet.py:170-183``): VALID conv + bias + ReLU.  A conv layer runs as the
  same typed GEMM over its NHWC im2col rows: row (sample, oh, ow), k = (kh, kw, cin) -- the TF kernel layout
  [kh, kw, cin, cout] of the parameter store is already that [K, Cout] matrix.  The im2col / col2im are
  torch views (``unfold``) and their autograd.

Each layer is one autograd node over the HIP kernels: fwd (out + ReLU mask [R][M][C]), dgrad (dX) and wgrad
(dW, db of every module, deterministic owners).  Widths <= 64 use the VALU kernels; wider layers (or
``set_mfma("always")``) use the fp32-MFMA kernels (``v_mfma_f32_16x16x4_f32``: exact fp32 products).
Rows are grouped by path: row r of a layer belongs to path ``r // rows_per_path``.  The numerics oracle is
``models.pathnet.trunk_forward_ref``.
"""
from __future__ import annotations

from typing import List

import torch

from . import _lib

_MFMA = "auto"          # "auto": MFMA when a layer is wider than 64 or M > 16; "always"; "never"


def set_mfma(mode: str):
    global _MFMA
    if mode not in ("auto", "always", "never"):
        raise ValueError(mode)
    _MFMA = mode


def _use_mfma(C: int) -> bool:
    return _MFMA == "always" or (_MFMA == "auto" and C > 64)


def _types(store) -> List[torch.Tensor]:
    cache = getattr(store, "_typed_fc_types", None)
    if cache is None:
        from ..models.pathnet import module_type
        cfg = store.cfg
        if cfg.M > 16:
            raise NotImplementedError("typed trunk: M <= 16")
        cache = []
        for l, spec in enumerate(cfg.layers):
            li = store.layout.layer_info[l]
            t = [module_type(spec, j) for j in range(cfg.M)]
            if spec.kind == "conv" and any(v != 1 for v in t):
                raise ValueError(f"layer {l}: conv modules are conv + ReLU only (type 1)")
            if spec.kind not in ("conv", "fc"):
                raise NotImplementedError(spec.kind)
            if any(v != 1 for v in t) and li["K"] != li["cout"]:
                raise ValueError(f"layer {l}: skip/residual modules need in width == out width")
            cache.append(torch.tensor(t, dtype=torch.int32, device=store.flat.device))
        store._typed_fc_types = cache
    return cache


class _TypedLayer(torch.autograd.Function):
    """One typed layer on [P * rpp, K] rows -> [P * rpp, C]; gradients for the flat store and the input."""

    @staticmethod
    def forward(ctx, flat, h, mask_l, store, l, rpp, need_dx):
        cfg = store.cfg
        li = store.layout.layer_info[l]
        K, C = li["K"], li["cout"]
        P = mask_l.shape[0]
        h = h.contiguous()
        _lib.check(h, torch.float32, shape=(P * rpp, K), name=f"x[{l}]")
        out = torch.empty(P * rpp, C, dtype=torch.float32, device=h.device)
        relu = torch.empty(P * rpp, cfg.M, C, dtype=torch.uint8, device=h.device)
        mfma = _use_mfma(C)
        _lib.call("launch_typed_fc_fwd_mfma" if mfma else "launch_typed_fc_fwd", h.data_ptr(), K, flat.data_ptr(),
                  li["offset"], li["chunk"], C, cfg.M, mask_l.data_ptr(), _types(store)[l].data_ptr(), P, rpp,
                  out.data_ptr(), relu.data_ptr(), _lib.stream())
        ctx.store, ctx.l, ctx.rpp, ctx.P, ctx.mfma, ctx.need_dx = store, l, rpp, P, mfma, need_dx
        ctx.save_for_backward(flat, h, mask_l, relu)
        return out

    @staticmethod
    def backward(ctx, gout):
        flat, h, mask_l, relu = ctx.saved_tensors
        store, l, rpp, P, mfma = ctx.store, ctx.l, ctx.rpp, ctx.P, ctx.mfma
        cfg = store.cfg
        li = store.layout.layer_info[l]
        K, C = li["K"], li["cout"]
        types = _types(store)[l]
        g = gout.contiguous().float()
        s = _lib.stream()
        gflat = torch.zeros_like(flat)
        _lib.call("launch_typed_fc_wgrad_mfma" if mfma else "launch_typed_fc_wgrad", h.data_ptr(), g.data_ptr(), K,
                  li["offset"], li["chunk"], C, cfg.M, P, mask_l.data_ptr(), types.data_ptr(), rpp, relu.data_ptr(),
                  gflat.data_ptr(), s)
        dx = None
        if ctx.need_dx:
            dx = torch.empty(P * rpp, K, dtype=torch.float32, device=g.device)
            _lib.call("launch_typed_fc_dgrad_mfma" if mfma else "launch_typed_fc_dgrad", g.data_ptr(), K,
                      flat.data_ptr(), li["offset"], li["chunk"], C, cfg.M, mask_l.data_ptr(), types.data_ptr(), P,
                      rpp, relu.data_ptr(), dx.data_ptr(), s)
        return gflat, dx, None, None, None, None, None


def im2col_nhwc(h: torch.Tensor, k: int, stride: int) -> torch.Tensor:
    """[B, H, W, C] -> [B * Ho * Wo, k * k * C] with k-order (kh, kw, c) (TF conv kernel layout)."""
    B, H, W, C = h.shape
    u = h.unfold(1, k, stride).unfold(2, k, stride)            # [B, Ho, Wo, C, kh, kw]
    Ho, Wo = u.shape[1], u.shape[2]
    return u.permute(0, 1, 2, 4, 5, 3).reshape(B * Ho * Wo, k * k * C), Ho, Wo


def typed_trunk_forward(store, x: torch.Tensor, mask_paths: torch.Tensor, rows_per_path: int) -> torch.Tensor:
    """x [P*rows_per_path, *input_shape] fp32 (NHWC for conv nets), mask_paths [P, L, M]
    -> features [P*rows_per_path, feature_dim].  Differentiable w.r.t. ``store.flat``."""
    cfg = store.cfg
    if cfg.trunk_scale == "M":
        raise NotImplementedError("typed trunk implements trunk_scale='none'")
    P = mask_paths.shape[0]
    B = x.shape[0]
    if B != P * rows_per_path:
        raise ValueError("x rows must equal P * rows_per_path")
    masks = mask_paths.float().contiguous()
    flat = store.flat
    h = x.float()
    for l, spec in enumerate(cfg.layers):
        li = store.layout.layer_info[l]
        ml = masks[:, l, :].contiguous()
        need_dx = l > 0 or x.requires_grad
        if spec.kind == "conv":
            cin = li["cin"]
            H = li["in_shape"][0]
            hs = h.reshape(B, H, -1, cin)
            cols, Ho, Wo = im2col_nhwc(hs, spec.kernel, spec.stride)
            y = _TypedLayer.apply(flat, cols, ml, store, l, rows_per_path * Ho * Wo, need_dx)
            h = y.reshape(B, Ho, Wo, li["cout"])
        else:
            h = _TypedLayer.apply(flat, h.reshape(B, -1), ml, store, l, rows_per_path, need_dx)
    return h.reshape(B, -1)
