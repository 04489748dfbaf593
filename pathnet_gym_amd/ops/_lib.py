"""ctypes binding of ``libpathnet_hip.so`` (the hand-written gfx950 kernels).

The library exports a plain C ABI: raw device pointers, scalars and a
``hipStream_t``.  It is loaded AFTER torch so that it binds to the HIP
runtime torch already loaded (same SONAME ``libamdhip64.so.7``): torch
tensors' ``data_ptr()`` and torch streams are valid handles for it, and
kernels launched on torch's current stream are captured by
``torch.cuda.graph`` (hipGraph) like any torch op.

No silent fallback: on a GPU box a missing library raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_float, c_int, c_long, c_uint, c_void_p, c_size_t

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "_hip", "libpathnet_hip.so")

P = c_void_p
_SIGS = {
    "launch_conv_fwd": [P, c_int, P, P, P, P, c_long, c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                        c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_long, c_float,
                        c_float, P],
    "launch_fc_fwd": [P, c_int, P, P, P, P, c_long, c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                      c_int, c_int, c_int, c_long, c_float, P],
    "launch_conv_wgrad": [P, c_int, P, P, P, c_long, c_long, c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int,
                          c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_long, c_int,
                          c_float, c_float, P],
    "launch_conv_dgrad": [P, P, P, c_long, c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                          c_int, c_int, c_int, c_int, c_int, c_int, c_long, c_float, P, P],
    "launch_fc_dgrad": [P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_long, c_float,
                        P, P, P],
    "launch_fc_wgrad_gm": [P, c_int, P, P, c_long, c_long, c_int, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int,
                           c_int, c_int, c_long, c_int, P],
    "launch_fc_wgrad": [P, c_int, P, P, P, c_long, c_long, c_int, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int,
                        c_int, c_int, c_long, c_float, P],
    "launch_heads_fwd_sample": [P, c_int, P, c_long, c_long, c_long, c_long, c_int, c_int, P, P, P, c_uint, P, c_int,
                                c_int, c_int, c_int, c_uint, P],
    "launch_a2c_grad": [P, P, P, P, P, P, c_int, c_int, c_int, c_float, c_float, c_float, c_float, c_float, c_float,
                        P, P, P, P],
    "launch_heads_bwd": [P, c_int, P, P, c_int, c_int, P, c_long, c_long, c_long, c_long, P, P, P],
    "launch_fitness_update": [P, P, c_int, c_int, c_int, P, P, P, P, c_int, P, P],
    "launch_rmsprop": [P, P, P, P, P, P, P, c_int, P, P, P, P, P, c_float, c_float, c_float, c_float, P],
    "launch_refresh_weights": [P, c_long, c_int, c_int, c_int, c_int, c_int, P, P, P],
    "launch_pong_step": [P, P, P, c_int, P, P, P, P, P, P, c_int, c_uint, c_int, c_int, c_int, c_int, c_int, c_int,
                         c_int, c_int, c_int, c_uint, P],
    "launch_refresh_weights_cmajor": [P, c_long, c_int, c_int, c_int, c_int, c_int, c_int, P, c_int, P],
    "fast_conv1_ring_fwd": [P, P, P, P, P, P, c_long, c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                            c_int, c_long, c_float, c_float, P, P, P],
    "fast_conv1_ring_wgrad": [P, P, P, P, P, c_long, c_long, c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int,
                              c_int, c_long, c_float, c_float, P],
    "launch_inv_group": [P, P, P, c_int, c_int, c_int, c_int, c_int, P, P, P, P],
    "launch_pong_step_ring": [P, P, P, c_int, P, c_long, P, P, P, P, P, P, c_int, c_uint, c_int, c_int, c_int, c_int,
                              c_int, c_int, c_int, c_int, c_uint, P],
    "launch_pong_heads_step_ring": [P, P, c_int, P, c_long, P, P, P, P, P, P, c_int, c_uint, c_int, c_int, c_int,
                                    c_int, c_int, c_int, c_int, c_int, c_uint, c_int, P, c_int, P, c_long, c_long,
                                    c_long, c_long, P, P, P, c_uint, P, c_int, c_int, c_uint, P],
    "launch_pong_step_ring_split": [P, P, P, c_int, P, c_long, P, P, P, P, P, P, c_int, c_uint, c_int, c_int, c_int,
                                    c_int, c_int, c_int, c_int, c_int, c_uint, c_int, c_int, P],
    "launch_cartpole_step": [P, P, P, P, P, c_int, c_uint, c_uint, c_int, P, P, P, P, P, P],
    "launch_pong_digit_tables": [P, c_int, c_int, c_int, c_int, c_int, P],
    "x3_refresh_weights_all": [P, c_int, P, P, P, c_int, c_int, P, P],
    "launch_opt_tail": [P, P, c_int, c_int, c_int, P, P, P, P, P, c_int, P, P, P, P],
    "pong_tables_ints": [],
    "launch_rgb_stack_push": [P, P, P, P, P, c_int, c_int, c_int, c_int, P],
    "launch_rects_stack_push": [P, P, c_int, c_int, P, P, P, P, c_int, P],
    "launch_rects_ring_push": [P, P, c_int, c_int, P, c_long, P, P, P, P, c_int, P],
    "launch_game_step": [c_int, P, P, P, c_int, c_int, c_int, c_uint, c_uint, c_int, c_int, P, P, P, P, P],
    "game_layout": [c_int, P, P],
    "fast_conv_fwd": [P, c_int, P, P, P, P, c_long, c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                      c_int, c_int, c_int, c_int, c_int, c_int, c_long, c_float, c_float, P, P, P],
    "launch_refresh_weights_f16": [P, c_long, c_int, c_int, c_int, c_int, c_int, P, P, P],
    "fast_conv_wgrad": [P, c_int, P, P, P, c_long, c_long, c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int,
                        c_int, c_int, c_int, c_int, c_int, c_int, c_long, c_float, c_float, P],
    "fast_conv_dgrad": [P, P, P, c_long, c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                        c_int, c_int, c_int, c_long, c_float, P, P],
    "launch_lstm_fwd": [P, c_int, P, P, P, P, P, c_long, P, P, P, P, c_int, c_int, c_int, P],
    "launch_lstm_bwd_point": [P, P, P, P, P, P, P, P, P, P, c_int, c_int, P],
    "launch_lstm_bwd_gemm": [P, P, P, c_int, P, c_int, c_int, c_int, P],
    "launch_lstm_wgrad": [P, P, P, c_long, c_long, c_int, c_int, c_long, c_int, P],
    "launch_lstm_refresh": [P, c_long, c_int, c_int, P, P, P],
    "launch_lstm_carry": [P, P, P, P, P, c_int, c_int, P],
    "launch_lstm_fwd_x3": [P, c_int, P, P, P, P, P, c_long, P, P, P, P, P, P, c_int, c_int, c_int, P],
    "launch_lstm_bwd_point_x3": [P, P, P, P, P, P, P, P, P, P, P, c_int, c_int, P],
    "launch_lstm_bwd_gemm_x3": [P, P, P, c_int, P, P, c_int, c_int, c_int, P],
    "launch_lstm_wgrad_x3": [P, P, P, c_long, c_long, c_int, c_int, c_long, c_int, P, c_int, P, P],
    "launch_lstm_refresh_x3": [P, c_long, c_int, c_int, P, P, P, P],
    "launch_lstm_carry_f32": [P, P, P, P, P, c_int, c_int, P],
    "fast_conv_set_slab": [c_int],
    "fast_conv_set_slab_fwd": [c_int],
    "fast_conv_set_dgrad_mfma": [c_int],
    "fast_conv_set_img_fwd": [c_int],
    "fast_conv_set_wgrad_ob": [c_int],
    "fast_conv_set_fwd_nt": [c_int],
    "fast_conv_set_wgrad_pf": [c_int],
    "fast_conv_set_f16_fwd": [c_int],
    "launch_ga_step": [P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_uint, P, P],
    "launch_ga_compact": [P, P, c_int, c_int, c_int, c_int, P, P, P, P, P, P, P],
    "launch_typed_fc_fwd": [P, c_int, P, c_long, c_long, c_int, c_int, P, P, c_int, c_int, P, P, P],
    "launch_typed_fc_dgrad": [P, c_int, P, c_long, c_long, c_int, c_int, P, P, c_int, c_int, P, P, P],
    "launch_typed_fc_wgrad": [P, P, c_int, c_long, c_long, c_int, c_int, c_int, P, P, c_int, P, P, P],
    "launch_typed_fc_fwd_mfma": [P, c_int, P, c_long, c_long, c_int, c_int, P, P, c_int, c_int, P, P, P],
    "launch_typed_fc_dgrad_mfma": [P, c_int, P, c_long, c_long, c_int, c_int, P, P, c_int, c_int, P, P, P],
    "launch_typed_fc_wgrad_mfma": [P, P, c_int, c_long, c_long, c_int, c_int, c_int, P, P, c_int, P, P, P],
    "launch_active_union": [P, P, c_int, c_int, c_int, P, P],
    "launch_prof_marker": [c_int, P],
    "launch_pack_ranges": [P, P, P, c_int, c_long, c_int, P],
    "launch_heads_fwd_sample_f32": [P, c_int, P, c_long, c_long, c_long, c_long, c_int, c_int, P, P, P, c_uint, P,
                                    c_int, c_int, c_int, c_int, c_uint, P],
    "launch_heads_bwd_f32": [P, c_int, P, P, c_int, c_int, P, c_long, c_long, c_long, c_long, P, P, P],
    "launch_conv_fwd_f32": [P, c_int, P, P, P, P, c_long, c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int,
                            c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_long,
                            c_float, c_float, P],
    "launch_fc_fwd_f32": [P, c_int, P, P, P, P, c_long, c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int,
                          c_int, c_int, c_int, c_int, c_long, c_float, P],
    "launch_conv_wgrad_f32": [P, c_int, P, P, P, P, c_long, c_long, c_int, P, P, P, P, P, c_int, c_int, c_int, c_int,
                              c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                              c_int, c_long, c_int, c_float, c_float, P],
    "launch_conv_dgrad_f32": [P, P, P, c_long, c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                              c_int, c_int, c_int, c_int, c_int, c_int, c_long, c_float, P, P],
    "launch_fc_dgrad_f32": [P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_long,
                            c_float, P, P],
    "launch_fc_wgrad_f32": [P, c_int, c_int, P, P, P, c_long, c_long, c_int, P, P, P, c_int, c_int, c_int, c_int, c_int,
                            c_int, c_int, c_int, c_long, c_float, P],
    "launch_refresh_weights_f32": [P, c_long, c_int, c_int, c_int, c_int, c_int, P, P, P],
    "launch_heads_bwd_det": [P, c_int, c_int, P, P, c_int, c_int, P, c_long, c_long, c_long, c_long, P, P, P, P],
    "heads_bwd_part_numel": [c_int, c_int, c_int],
    "heads_bwd_split_numel": [c_int, c_int, c_int],
    "launch_heads_bwd_split": [P, c_int, c_int, P, P, c_int, c_int, P, c_long, c_long, c_long, c_long, P, P, P, P],
    "fast_conv_dgrad_bf16": [P, c_int, P, P, c_long, c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                             c_int, c_int, c_int, c_int, c_int, c_long, c_float, P, c_int, P],
    "fast_conv_wgrad_bf16g": [P, c_int, P, P, P, c_long, c_long, c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int,
                              c_int, c_int, c_int, c_int, c_int, c_int, c_long, c_float, c_float, P],
    "x3_conv_fwd": [P, c_long, c_int, P, c_long, P, P, c_long, P, c_long, c_int, P, P] + [c_int] * 13
                   + [c_long, c_float, c_float, P],
    "x3_conv_wgrad": [P, c_long, c_int, P, P, P, c_long, c_long, c_int, P, P] + [c_int] * 12
                     + [c_long, c_float, c_float, P, P],
    "x3_conv1_ring_fwd": [P, P, P, c_long, P, P, c_long, P, c_long, c_int, P, P] + [c_int] * 8
                         + [c_long, c_float, c_float, P],
    "x3_conv23_fwd": [P, c_long, P, c_long, P, c_long, P, c_long, c_long, c_int, P, c_long, P, c_long, P, c_long,
                      c_long, c_int, P, P, P] + [c_int] * 7 + [c_float, c_float, P],
    "x3_conv1_ring_wgrad": [P, P, P, P, P, c_long, c_long, c_int, P, P] + [c_int] * 7 + [c_long, c_float, c_float, P,
                                                                                         P],
    "x3_conv_dgrad": [P, P, P, c_long, c_int, P, P] + [c_int] * 12 + [c_long, c_float, P, P, P, P],
    "x3_fc_fwd": [P, c_long, c_int, P, c_long, P, P, c_long, P, c_long, c_int, P, P] + [c_int] * 10
                 + [c_long, c_float, P],
    "x3_fc_heads_fwd": [P, c_long, c_int, P, P, P, c_long, P, c_long, c_int, P, P] + [c_int] * 9
                       + [c_long, c_float, c_long, c_long, c_long, c_long, c_int, P, P, P, c_uint, P, c_int, c_int,
                          c_int, c_uint, P],
    "x3_fc_fwd_mm": [P, c_long, c_int, P, c_long, P, P, c_long, P, c_long, c_int, P, P, P, P, P, P] + [c_int] * 10
                    + [c_long, c_float, P],
    "x3_fc_dgrad": [P, P, P, c_long, P, P] + [c_int] * 9 + [c_long, c_float, P, P, c_long, P, P, P],
    "x3_amax": [P, c_long, P, P],
    "x3_amax_reset": [P, c_int, P],
    "x3_fc_wgrad_gm": [P, c_long, c_int, P, c_long, P, c_long, c_long, c_int, P, P, P] + [c_int] * 8
                      + [c_long, c_int, P, P],
    "x3_fc_wgrad": [P, c_long, c_int, P, P, P, c_long, c_long, c_int, P, P, P] + [c_int] * 8 + [c_long, c_float, P, P],
    "x3_refresh_weights": [P, c_long, c_int, c_int, c_int, c_int, c_int, P, P, c_int, P, P],
    "x3_status_fold": [P, P, P],
    "x3_set_fx": [P],
    "x3_fx_flush": [P, P, c_long, c_long, P],
    "fast_conv_set_x3_fwd_nt": [c_int],
    "fast_conv_set_x3_fwd_lb": [c_int],
    "fast_conv_set_x3_fwd_db": [c_int],
    "fast_conv_set_x3_fwd_sw": [c_int],
    "fast_conv_set_x3_wg3_tile": [c_int],
    "fast_conv_set_x3_fc_mmv": [c_int],
    "fast_conv_set_x3_fc_dg_gemm": [c_int],
    "fast_conv_set_x3_fcw_kt": [c_int],
    "fast_conv_set_x3_dg_w3": [c_int],
    "fast_conv_set_x3_c1_f16b": [c_int],
    "fast_conv_set_x3_dg_fold": [c_int],
    "fast_conv_set_x3_fwd_tile": [c_int],
    "fast_conv_set_x3_c1_band": [c_int],
    "fast_conv_set_x3_c1_pipe": [c_int],
    "heads_set_s16": [c_int],
    "heads_set_bwd_rows": [c_int],
    "fast_conv_set_x3_fc_d": [c_int],
    "fast_conv_set_x3_fc_ks": [c_int],
    "fast_conv_set_x3_wgrad_pf": [c_int],
    "fast_conv_set_x3_c1_wg_ncx": [c_int],
    "fast_conv_set_x3_wg_target": [c_int],
    "fast_conv_set_x3_wg_auto": [c_int],
    "fast_conv_set_x3_wg2_target": [c_int],
    "fast_conv_set_x3_wg3_target": [c_int],
    "fast_conv_set_x3_c1f_target": [c_int],
    "fast_conv_set_x3_fc_rt1": [c_int],
    "fast_conv_set_x3_c1f_minb": [c_int],
    "fast_conv_set_x3_c23_target": [c_int],
    "fast_conv_set_x3_c23_mins": [c_int],
    "fast_conv_set_x3_fcw_target": [c_int],
    "fast_conv_set_x3_dg3_target": [c_int],
    "fast_conv_set_x3_slab_pmap": [c_int],
    "fast_conv_set_x3_c1_sb1": [c_int],
    "fast_conv_set_x3_presplit": [c_int],
    "fast_conv_set_x3_fh_d": [c_int],
    "fast_conv_set_x3_dg_target": [c_int],
    "fast_conv_set_x3_fc_ks_parts": [c_int],
    "conv_fwd_smem": [c_int, c_int],
    "conv_wgrad_smem": [c_int],
}

_lib = None


def available() -> bool:
    return os.path.exists(LIB_PATH)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"HIP kernel library missing at {LIB_PATH}; run `python -m pathnet_gym_amd._build`")
        _lib = ctypes.CDLL(LIB_PATH)
        for name, args in _SIGS.items():
            fn = getattr(_lib, name)
            fn.argtypes = args
            fn.restype = c_size_t if name.endswith("_smem") else c_long if name.endswith("_numel") else (None if name.startswith("fast_conv_set_") else c_int)
    return _lib


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t) -> int:
    if t is None:
        return None
    return t.data_ptr()


def call(name: str, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed with code {rc}")


def call_fast(name: str, *args) -> bool:
    """Specialised-shape launcher: True if it handled the call, False if the shape is not specialised."""
    rc = getattr(lib(), name)(*args)
    if rc < 0:
        raise RuntimeError(f"{name} failed with code {rc}")
    return rc == 1


USE_FAST = True


def check(t: torch.Tensor, dtype=None, shape=None, numel=None, name="tensor", cuda=True):
    """Host-side validation before any launch (a bad shape must never reach a kernel)."""
    if cuda and t.device.type != "cuda":
        raise ValueError(f"{name} must be on the GPU")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"{name}: dtype {t.dtype} != {dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: shape {tuple(t.shape)} != {tuple(shape)}")
    if numel is not None and t.numel() < numel:
        raise ValueError(f"{name}: numel {t.numel()} < required {numel}")
    return t
