"""HIP PathNet trunk: geometry, bf16 MFMA operand copies, per-layer launches.

Buffers (all device, B = P*E, slots = T+1 steps so the bootstrap forward can
reuse them):

=============  =========================================  ==================
name           layout                                     written by
=============  =========================================  ==================
obs            [T+1][B][H*W*C] uint8 (pixels) or           env step kernel
               [T+1][B][8] bf16 (vector envs)
frames, fc     frame ring [B][T+4][H*W] uint8 + first valid    ring env step
               channel [T+1][B] (replaces obs for Pong)
acts[l]        [T+1][B][HWo*Cout] bf16 (module-sum out)    fwd epilogue
bits[l] conv   [M][(T+1)*B*HWo] uint8 (8 maps/byte)        fwd epilogue
bits[l] fc     [M][(T+1)*B][Cout/16] uint16                fwd epilogue
grads[l]       [T*B][HWo*Cout] fp32 (dL/d acts[l])         dgrad of l+1 /
                                                           heads_bwd (l=L-1)
Wc[l]          [M][Cout][KP] bf16  (B operand, fwd)        refresh kernel
WcT[l] (fc)    [M][KP][Cout] bf16  (B operand, fc dgrad)   refresh kernel
=============  =========================================  ==================

``bits`` rows are indexed by GLOBAL row (sample_global*HWo + pos) so the
forward of step t and the whole-rollout backward agree.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch

from . import _lib


def round_up(x, m):
    return (x + m - 1) // m * m


# -- fp32x activation storage (csrc/trunk_x3.hip): an activation between layers is kept as its fp16 pair in two
# 16-bit planes of one [2, ...] allocation (hi + lo == the fp32 value to 2^-22; the weight-gradient kernels convert it
# to the bf16 pair while staging).  The tensor handle is plane 0 (fp16 hi); plane 1 of any view starts one plane
# length further on.
def x2_alloc(shape, device) -> torch.Tensor:
    """Plane 0 (fp16 hi) of a zeroed [2, *shape] fp16-pair allocation."""
    return torch.zeros((2,) + tuple(shape), dtype=torch.float16, device=device)[0]


def x2_lo(t: torch.Tensor) -> int:
    """Elements from any element of plane 0 of a pair tensor to the same element of plane 1 (plane length)."""
    nb = t.untyped_storage().nbytes()
    if t.dtype != torch.float16 or nb % 4 != 0 or t.storage_offset() + t.numel() > nb // 4:
        raise ValueError("not plane 0 of a fp16-pair allocation (x2_alloc)")
    return nb // 4


def _plane(t: torch.Tensor, k: int, dtype) -> torch.Tensor:
    v = torch.empty(0, dtype=torch.float16, device=t.device).set_(t.untyped_storage(), t.storage_offset() + k * x2_lo(t),
                                                                 t.size(), t.stride())
    return v if dtype == torch.float16 else v.view(dtype)


def x2_value(t: torch.Tensor) -> torch.Tensor:
    """fp32 value hi + lo of an fp16-pair tensor."""
    return t.float() + _plane(t, 1, torch.float16).float()


@dataclass
class LayerGeom:
    kind: str
    K: int
    KP: int
    Cout: int
    HWo: int
    out_feat: int
    w_off: int
    chunk: int
    Hin: int = 1
    Win: int = 1
    Cin: int = 1
    KH: int = 1
    KW: int = 1
    S: int = 1
    Ho: int = 1
    Wo: int = 1
    ldx: int = 0            # fc input row stride
    u8in: bool = False
    in_scale: float = 1.0

    @property
    def b_off(self):
        return self.w_off + self.K * self.Cout


# conv geometries with fp32x kernels (csrc/trunk_x3.hip): (Hin, Win, Cin, kernel, stride, uint8 input)
X3_CONV_GEOMS = ((160, 120, 4, 8, 4, True), (39, 29, 8, 4, 2, False), (18, 13, 8, 3, 1, False))


def x3_unsupported_reason(net) -> Optional[str]:
    """Why the fp32x kernels cannot run PathNetConfig ``net`` (None: they can).  The trainer then runs the fp32 engine
    (csrc/trunk_f32.hip: fp32 operands, at least the accuracy fp32x promises, bit-reproducible, slower) instead of
    failing -- e.g. for the reference's --kernel_num / --stride_size flags beyond the default 8,4,3 / 4,2,1 trunk."""
    if net.M > 10:
        return f"M={net.M} > 10 modules per layer"
    for l, (spec, (ins, outs, K, cin)) in enumerate(zip(net.layers, net.layer_shapes())):
        if spec.kind == "conv":
            g = (ins[0], ins[1], ins[2], spec.kernel, spec.stride, l == 0)
            if g not in X3_CONV_GEOMS:
                return f"conv layer {l} geometry {g[:5]} has no fp32x kernel"
        elif l == 0 or spec.out % 64 != 0 or K % 8 != 0:
            return f"fc layer {l} needs a conv input and width % 64 == 0"
    return None


class HipPathNet:
    """Kernel-side view of an ``ACPathNet`` (created by it when backend='hip')."""

    # wide fc layers take their weight gradient from the masked bf16 gradient the dgrad kernel
    # writes (fc_wgrad_gm_kernel); PATHNET_FC_WGRAD_GM=0 selects the fp32-G tile kernel (A/B)
    fc_wgrad_gm = os.environ.get("PATHNET_FC_WGRAD_GM", "1") != "0"
    fc_wgrad_gm_min_k = int(os.environ.get("PATHNET_FC_WGRAD_GM_MIN_K", "1024"))

    def __init__(self, model):
        if not torch.cuda.is_available():
            raise RuntimeError("HIP backend requested but no GPU is visible")
        _lib.lib()   # fail loudly if the library is missing
        self.model = model
        cfg = model.cfg
        self.cfg = cfg
        # compute_dtype "fp32": fp32 activations / operand copies on v_mfma_f32_16x16x4_f32 (csrc/trunk_f32.hip,
        # every reduction in a fixed order); "bf16": the bf16/fp16-operand MFMA kernels with fp32 accumulation
        self.f32 = getattr(model, "compute_dtype", "bf16") == "fp32"
        # compute_dtype "fp32x": fp32-accurate split-bf16 operands (csrc/trunk_x3.hip): every activation between
        # layers is a (hi, lo) bf16 pair, every MFMA product hi*hi + hi*lo + lo*hi, the last layer's output fp32
        self.x3 = getattr(model, "compute_dtype", "bf16") == "fp32x"
        # fp32x, deterministic: every weight-gradient contribution that would meet others in an fp32 atomic is added
        # as an int64 fixed-point number instead (csrc/common.h gacc: integer addition is associative, so the
        # arrival order of workgroups and waves no longer matters) and converted back once per backward
        # (x3_fx_flush); the routing (frame ring, fused LSTM, split heads backward -- already fixed-order) is the
        # default fp32x one
        self.fx_det = self.x3 and bool(getattr(model, "deterministic", False))
        self._fxbuf = None
        if self.fx_det:
            n = model.store.layout.numel
            self._fxbuf = torch.zeros(n + 1, dtype=torch.int64, device=model.device)   # [0]: range guard word
        self.act_dtype = torch.float32 if self.f32 else torch.bfloat16
        # deterministic reductions (TrainConfig.deterministic; implied by fp32): every weight/bias gradient is
        # summed in a fixed order (trunk_f32.hip ordered slabs, heads_reduce_kernel) instead of fp32 atomics,
        # so one seed reproduces the update bit for bit
        self.deterministic = self.f32 or (bool(getattr(model, "deterministic", False)) and not self.x3)
        self._hpart = None
        self._hsplit = None
        self.L, self.M = cfg.L, cfg.M
        lay = model.store.layout
        dev = model.device
        self.geoms: List[LayerGeom] = []
        for l, (spec, li) in enumerate(zip(cfg.layers, lay.layer_info)):
            ins, outs = li["in_shape"], li["out_shape"]
            K, cout = li["K"], li["cout"]
            if spec.kind == "conv":
                Hin, Win, Cin = ins
                Ho, Wo, _ = outs
                if Cin not in (4, 8) and not (l == 0):
                    raise NotImplementedError("conv layers need Cin in {4, 8}")
                if cout != 8:
                    raise NotImplementedError("HIP conv modules have 8 output maps (reference feature_num)")
                g = LayerGeom("conv", K, round_up(K, 32), cout, Ho * Wo, Ho * Wo * cout, li["offset"], li["chunk"],
                              Hin, Win, Cin, spec.kernel, spec.kernel, spec.stride, Ho, Wo,
                              u8in=(l == 0), in_scale=(1.0 / 255.0 if l == 0 else 1.0))
                if l == 0 and (Cin * 2) % 8 != 0:
                    raise NotImplementedError("first conv layer needs Cin*KW multiple of 8 bytes")
            else:
                if spec.module_types is not None and any(t != 1 for t in spec.module_types):
                    raise NotImplementedError("HIP fc layers implement fc+ReLU modules")
                if cout % 32 != 0:
                    raise NotImplementedError("HIP fc modules need width % 32 == 0")
                ldx = round_up(K, 8) if l > 0 else (K if self.f32 else 8)
                if l == 0 and K > 8:
                    raise NotImplementedError("vector observations up to 8 dims")
                g = LayerGeom("fc", K, round_up(K, 32), cout, 1, cout, li["offset"], li["chunk"], ldx=ldx)
                if l > 0 and self.geoms[-1].out_feat != K:
                    raise ValueError("fc input size mismatch")
                if l > 0 and K % 8 != 0:
                    raise NotImplementedError("HIP fc layers need input width % 8 == 0")
            self.geoms.append(g)
        self.pixels = cfg.layers[0].kind == "conv"
        self.out_scale_last = (1.0 / cfg.M) if cfg.trunk_scale == "M" else 1.0
        if self.x3:
            self._check_x3()
        # MFMA operand copies (bf16, or fp32 in the fp32 mode; fp32x: [2, ...] hi/lo planes, the uint8 first
        # layer's as the fp16 pair of W * 2^8)
        self.Wc = []
        self.WcT = []
        npl = (2,) if self.x3 else ()
        for l, g in enumerate(self.geoms):
            wdt = torch.float16 if self.x3 else self.act_dtype
            self.Wc.append(torch.zeros(npl + (self.M, g.Cout, g.KP), dtype=wdt, device=dev))
            need_t = g.kind == "fc" and l > 0
            # fp32x: fp16 pieces of W^T * 2^8 (the fc input gradient's B operand against scaled fp16-pair gradients):
            # hi, lo and the third piece (the residual W - hi - lo, csrc/trunk_x3.hip X3_DG_W3)
            self.WcT.append(torch.zeros(((3,) if self.x3 else ()) + (self.M, g.KP, g.Cout),
                                        dtype=torch.float16 if self.x3 else self.act_dtype, device=dev)
                            if need_t else None)
        self.x3_status = torch.zeros(1, dtype=torch.int32, device=dev)   # fp16 range overflow of the scaled conv1 pair
        # fp32x backward: amax of every layer's output gradient (G16 scales, csrc/trunk_x3.hip g16_scale); layer L-1's
        # is measured when a backward starts, the others written by the input-gradient kernels of the layer above
        self.gamax = torch.zeros(max(1, len(cfg.layers)), dtype=torch.float32, device=dev)
        self._part = None            # fp32 conv wgrad partial slabs (allocated on first use, before capture)
        self._ys = None              # fp32x module-major fc forward: per-slot fp32 output planes
        # fp32x fc forward: module-major (csrc/trunk_x3.hip fc_fwd_mm2_x3: one workgroup per module x 128 rows of
        # its paths x 128 columns, LDS-staged tiles, then fc_slot_sum_x3) instead of path-major (fc_fwd_x3, which
        # re-reads a module's weights per path and is bound by its fragment loads).  The first module-major kernel
        # (register fragments, fast_conv_set_x3_fc_mmv(1)) measured slower (fc1 95.6 vs 70.3 us,
        # profiles/r3/kwin_x3_v6*.md).  PATHNET_X3_FC_MM=0 selects path-major.
        self.fc_fwd_mm = os.environ.get("PATHNET_X3_FC_MM", "1") == "1"
        self.fc_fwd_mm_min_k = int(os.environ.get("PATHNET_X3_FC_MM_MIN_K", "1024"))   # fc2 (K = 256): path-major
        # ... unless the launch is small (P*T*E rows <= this; measured at 8 paths: module-major k-split 4 + slot sum
        # 10.1 + 6.2 us vs path-major 16.2 us -- a wash, so off by default)
        self.fc_fwd_mm_small_rows = int(os.environ.get("PATHNET_X3_FC_MM_SMALL_ROWS", "0"))
        # conv2 + conv3 forward in one launch per rollout step (conv23_fwd)
        self.fuse23 = os.environ.get("PATHNET_X3_FUSE23", "1") != "0"
        # the last fc layer + heads + sampling of a rollout step in one launch (fc_heads_fwd): bit-identical but
        # measured slower (42 us vs 25 us for fc_fwd_x3 + heads at 64 and at 8 paths, scripts/diag/ab_kernel.py: one
        # wave walks every module of its 64 columns in turn, where fc_fwd_x3 gives each module its own wave and each
        # column tile its own workgroup), so off; PATHNET_X3_FUSE_HEADS=1 turns it on
        self.fuse_heads = os.environ.get("PATHNET_X3_FUSE_HEADS", "0") == "1"
        # target workgroup count of the fc1 weight gradient (paths split over ~wgs / tiles groups); at <= 16 paths a
        # split holds too few paths and 256 wins (8 paths: 173 -> 163 us), at 64 paths 768 (933 vs 1023 us at 256)
        self.fc_wgrad_gm_wgs = int(os.environ.get("PATHNET_X3_FC_WGRAD_WGS", "768"))
        self.fc_wgrad_gm_wgs_small = int(os.environ.get("PATHNET_X3_FC_WGRAD_WGS_SMALL", "256"))
        P = model.P
        self.inv_path = torch.zeros(self.L, self.M, P, dtype=torch.int32, device=dev)
        self.inv_slot = torch.zeros(self.L, self.M, P, dtype=torch.int32, device=dev)
        self.inv_cnt = torch.zeros(self.L, self.M, dtype=torch.int32, device=dev)
        # split rollout (runtime/engine.py rollout groups): per path group (p0, np), the group's own inverse lists
        # (group-local path indices, rebuilt on device at the start of every rollout) and fc slot planes
        self._groups = {}
        lay_h = lay.heads
        self.heads_off = lay_h
        # fused LSTM cell: csrc/lstm.hip (bf16 copies of the fp32 master kernel) or, in fp32x, csrc/lstm_x3.hip (fp16
        # hi+lo pairs, fp32 state: the reference's default network at its precision).  fp32 (deterministic) keeps
        # the hybrid autograd LSTM.
        self.lstm = None
        if cfg.use_lstm and not self.deterministic:
            ls = lay.lstm
            F, H = ls["din"], ls["H"]
            if F % 64 == 0 and H % 64 == 0:
                pl = (2,) if self.x3 else ()
                self.lstm = dict(F=F, H=H, k_off=ls["kernel"], b_off=ls["bias"], x3=self.x3,
                                 KpT=torch.zeros(pl + (4 * H, F + H), dtype=torch.float16 if self.x3 else torch.bfloat16,
                                                 device=dev),
                                 Kb=torch.zeros(pl + (F + H, 4 * H), dtype=torch.float16 if self.x3 else torch.bfloat16,
                                                device=dev),
                                 # fp32x G16 scales: [0] amax of the saved [x | h] rows, [1 + t] amax of step t's dz
                                 amax=torch.zeros(2, dtype=torch.float32, device=dev) if self.x3 else None)
        # frame-ring input for the first layer (runtime/engine.py): channel-major bf16 weights; fp32x reads the ring
        # into its packed LDS band / slab (csrc/trunk_x3.hip RING) and keeps its own weight pairs
        g0 = self.geoms[0]
        self.ring_ok = (not self.deterministic and not self.f32 and g0.kind == "conv" and g0.u8in and (g0.Hin, g0.Win, g0.Cin, g0.KH, g0.S) == (160, 120, 4, 8, 4)
                        and self.M <= 10 and g0.Cout == 8)
        self.Wc_ring = None
        # uint8 first conv layer: fp16 operand copy + per-column weight sums for the fp16-offset MFMA path
        # (conv_fwd_fast: pixels enter as fp16(1024 + v), built with one v_perm per two pixels)
        self.Wh0 = self.hcorr0 = None
        if g0.kind == "conv" and g0.u8in and not self.f32 and not self.x3:
            self.Wh0 = torch.zeros(self.M, g0.Cout, g0.KP, dtype=torch.float16, device=dev)
            self.hcorr0 = torch.zeros(self.M * g0.Cout, dtype=torch.float32, device=dev)
        self.refresh_weights()

    def enable_ring(self):
        """Allocate the channel-major first-layer weight copy used with the frame ring."""
        if not self.ring_ok:
            raise NotImplementedError("frame ring needs the 160x120x4 / 8x8 s4 first conv layer and M <= 10")
        if self.Wc_ring is None and not self.x3:
            g = self.geoms[0]
            dev = self.model.device
            self.Wc_ring = torch.zeros(self.M, g.Cout, g.KP, dtype=torch.bfloat16, device=dev)
            self.Wh_ring = torch.zeros(self.M, g.Cout, g.KP, dtype=torch.float16, device=dev)     # fp16-offset path
            self.refresh_weights()

    _X3_CONV = X3_CONV_GEOMS

    def _check_x3(self):
        """fp32x kernels exist for the reference pixel trunk geometries (csrc/trunk_x3.hip): uint8 160x120x4 8x8/s4,
        then 39x29x8 4x4/s2 and 18x13x8 3x3/s1 conv layers, fc layers of 64k outputs over >= 8-aligned inputs."""
        if self.M > 10:
            raise NotImplementedError("fp32x kernels hold up to 10 modules per layer")
        for l, g in enumerate(self.geoms):
            if g.kind == "conv":
                if (g.Hin, g.Win, g.Cin, g.KH, g.S, g.u8in) not in self._X3_CONV or g.u8in != (l == 0):
                    raise NotImplementedError(f"fp32x: conv layer {l} geometry {(g.Hin, g.Win, g.Cin, g.KH, g.S)} "
                                              "has no split-bf16 kernel")
            elif l == 0 or g.Cout % 64 != 0 or g.ldx % 8 != 0:
                raise NotImplementedError(f"fp32x: fc layer {l} needs a conv input and width % 64 == 0")

    def alloc_act(self, l: int, shape) -> torch.Tensor:
        """Output buffer of layer l: bf16 (bf16 mode), fp32 (fp32 mode, and the last layer in fp32x), or the hi plane
        of a split-bf16 pair (fp32x, between layers)."""
        dev = self.model.device
        if self.x3 and l < self.L - 1:
            return x2_alloc(shape, dev)
        dt = torch.float32 if (self.f32 or self.x3) else torch.bfloat16
        return torch.zeros(tuple(shape), dtype=dt, device=dev)

    @property
    def feat_dtype(self):
        return torch.float32 if (self.f32 or self.x3) else torch.bfloat16

    # ------------------------------------------------------------------
    def set_paths(self, expressed: np.ndarray):
        """Inverse module lists for the module-major fc wgrad (in place)."""
        P, L, M = expressed.shape
        ip = np.zeros((L, M, P), np.int32)
        isl = np.zeros((L, M, P), np.int32)
        ic = np.zeros((L, M), np.int32)
        for p in range(P):
            for l in range(L):
                act = np.nonzero(expressed[p, l] > 0.5)[0]
                for a, j in enumerate(act):
                    ip[l, j, ic[l, j]] = p
                    isl[l, j, ic[l, j]] = a
                    ic[l, j] += 1
        self.inv_path.copy_(torch.from_numpy(ip))
        self.inv_slot.copy_(torch.from_numpy(isl))
        self.inv_cnt.copy_(torch.from_numpy(ic))

    def set_frozen(self, frozen):
        pass   # frozen segments are skipped by the optimizer; kernels compute their grads (cheap)

    @property
    def reproducible(self) -> bool:
        """One seed reproduces every update bit for bit (fp32 engine, bf16 ordered reductions, fp32x fixed point)."""
        return bool(self.deterministic or self.fx_det)

    def fx_begin(self):
        """Deterministic fp32x: route the weight-gradient launches that follow into the fixed-point accumulator."""
        if self.fx_det:
            _lib.call("x3_set_fx", self._fxbuf.data_ptr() + 8)

    def fx_end(self, grad_flat: torch.Tensor, n0: int = 0, n1: Optional[int] = None):
        """... stop routing, and add the accumulated [n0, n1) into grad_flat (re-zeroing the accumulator)."""
        if not self.fx_det:
            return
        _lib.call("x3_set_fx", None)
        n1 = grad_flat.numel() if n1 is None else n1
        _lib.check(grad_flat, torch.float32, numel=self._fxbuf.numel() - 1, name="grad_flat")
        _lib.call("x3_fx_flush", self._fxbuf.data_ptr() + 8, grad_flat.data_ptr(), n0, n1, _lib.stream())

    def fold_x3_status(self, out: torch.Tensor):
        """fp32x: out[0] <- the fp16-pair range flags of the last rollout / weight refresh (csrc/trunk_x3.hip
        x3_status_fold; 0.0 = in range); the flags reset.  Graph-capturable (one tiny kernel)."""
        _lib.check(out, torch.float32, numel=1, name="status out")
        _lib.call("x3_status_fold", self.x3_status.data_ptr(), out.data_ptr(), _lib.stream())

    def check_x3_status(self, update: int = -1):
        """Host check of the fp16-pair range flags (syncs); raises runtime.guard.X3RangeError when set."""
        if not self.x3:
            return 0
        from ..runtime.guard import X3RangeError
        out = torch.zeros(1, dtype=torch.float32, device=self.model.device)
        self.fold_x3_status(out)
        v = float(out.item())
        if v != 0.0:
            raise X3RangeError(v, update)
        return 0

    def refresh_weights(self):
        flat = self.model.store.flat
        if self.x3:
            # every layer's fp16-pair copies in one launch (csrc/trunk_x3.hip x3_refresh_weights_all): the
            # descriptor arrays are built once (static buffer addresses)
            if getattr(self, "_refresh_args", None) is None:
                n = len(self.geoms)
                meta = (ctypes.c_long * (5 * n))(*[v for g in self.geoms for v in (g.w_off, g.chunk, g.K, g.KP, g.Cout)])
                wc = (ctypes.c_void_p * n)(*[self.Wc[l].data_ptr() for l in range(n)])
                wct = (ctypes.c_void_p * n)(*[_lib.ptr(self.WcT[l]) or None for l in range(n)])
                self._refresh_args = (n, meta, wc, wct)
            n, meta, wc, wct = self._refresh_args
            _lib.call("x3_refresh_weights_all", flat.data_ptr(), n, meta, wc, wct, self.M, 1,
                      self.x3_status.data_ptr(), _lib.stream())
            if self.lstm is not None:
                ls = self.lstm
                _lib.call("launch_lstm_refresh_x3", flat.data_ptr(), ls["k_off"], ls["F"], ls["H"], ls["KpT"].data_ptr(),
                          ls["Kb"].data_ptr(), self.x3_status.data_ptr(), _lib.stream())
            return
        for l, g in enumerate(self.geoms):
            _lib.call("launch_refresh_weights_f32" if self.f32 else "launch_refresh_weights", flat.data_ptr(), g.w_off, g.chunk, g.K, g.KP, g.Cout, self.M,
                      self.Wc[l].data_ptr(), _lib.ptr(self.WcT[l]), _lib.stream())
        if self.Wh0 is not None:
            g = self.geoms[0]
            _lib.call("launch_refresh_weights_f16", flat.data_ptr(), g.w_off, g.chunk, g.K, g.KP, g.Cout, self.M,
                      self.Wh0.data_ptr(), self.hcorr0.data_ptr(), _lib.stream())
        if self.Wc_ring is not None:
            g = self.geoms[0]
            for buf, f16 in ((self.Wc_ring, 0), (self.Wh_ring, 1)):
                _lib.call("launch_refresh_weights_cmajor", flat.data_ptr(), g.w_off, g.chunk, g.KH, g.KW, g.Cin,
                          g.Cout, self.M, buf.data_ptr(), f16, _lib.stream())
        if self.lstm is not None:
            ls = self.lstm
            _lib.call("launch_lstm_refresh", flat.data_ptr(), ls["k_off"], ls["F"], ls["H"], ls["KpT"].data_ptr(),
                      ls["Kb"].data_ptr(), _lib.stream())

    # -- fused LSTM cell (csrc/lstm.hip) ------------------------------------------
    @property
    def lstm_dtype(self):
        """dtype of the LSTM hidden state / saved [x | h] rows: fp32 in fp32x, bf16 otherwise."""
        return torch.float32 if self.x3 else torch.bfloat16

    def lstm_prepare(self, T: int):
        """fp32x: size the G16 amax slots for a T-step rollout (before any graph capture)."""
        ls = self.lstm
        if ls is not None and ls["x3"] and ls["amax"].numel() < T + 1:
            ls["amax"] = torch.zeros(T + 1, dtype=torch.float32, device=ls["amax"].device)

    def lstm_amax_reset(self):
        """fp32x: zero the G16 amaxes at the start of a rollout (the forward's xh rows, then the backward's dz)."""
        if self.lstm is not None and self.lstm["x3"]:
            self.lstm["amax"].zero_()

    def lstm_fwd(self, x, hprev, cprev, prev_done, hout, cout, gates=None, xh=None):
        """x [B,F], hprev [B,H] (bf16; fp32 in fp32x), cprev [B,H] f32, prev_done [B] u8 or None -> hout/cout
        (/gates/xh)."""
        ls = self.lstm
        B = x.shape[0]
        dt = self.lstm_dtype
        _lib.check(x, self.feat_dtype, name="lstm x")
        for t, nm in ((hprev, "hprev"), (hout, "hout")):
            _lib.check(t, dt, numel=B * ls["H"], name=nm)
        if xh is not None:
            _lib.check(xh, dt, numel=B * (ls["F"] + ls["H"]), name="xh")
        if ls["x3"]:
            _lib.call("launch_lstm_fwd_x3", x.data_ptr(), x.shape[1], hprev.data_ptr(), cprev.data_ptr(),
                      _lib.ptr(prev_done), ls["KpT"].data_ptr(), self.model.store.flat.data_ptr(), ls["b_off"],
                      hout.data_ptr(), cout.data_ptr(), _lib.ptr(gates), _lib.ptr(xh), self.x3_status.data_ptr(),
                      ls["amax"].data_ptr(), ls["F"], ls["H"], B, _lib.stream())
            return
        _lib.call("launch_lstm_fwd", x.data_ptr(), x.shape[1], hprev.data_ptr(), cprev.data_ptr(),
                  _lib.ptr(prev_done), ls["KpT"].data_ptr(), self.model.store.flat.data_ptr(), ls["b_off"],
                  hout.data_ptr(), cout.data_ptr(), _lib.ptr(gates), _lib.ptr(xh), ls["F"], ls["H"], B,
                  _lib.stream())

    def lstm_bwd_step(self, dh_heads, dh_rec, dc_rec, done_t, gates, c_t, c_prev, prev_done, dz, dc_out, dx,
                      dh_prev, t: int = 0):
        """One reverse step; t = the rollout step (fp32x: its dz amax slot, csrc/lstm_x3.hip G16)."""
        ls = self.lstm
        B = dh_heads.shape[0]
        st = _lib.stream()
        if ls["x3"]:
            if not 0 <= t < ls["amax"].numel() - 1:
                raise ValueError(f"lstm_bwd_step: step {t} has no amax slot (lstm_prepare({t + 1}) first)")
            am = ls["amax"].data_ptr() + 4 * (1 + t)
            _lib.call("launch_lstm_bwd_point_x3", dh_heads.data_ptr(), _lib.ptr(dh_rec), _lib.ptr(dc_rec),
                      _lib.ptr(done_t), gates.data_ptr(), c_t.data_ptr(), c_prev.data_ptr(), _lib.ptr(prev_done),
                      dz.data_ptr(), dc_out.data_ptr(), am, ls["H"], B, st)
            _lib.call("launch_lstm_bwd_gemm_x3", dz.data_ptr(), ls["Kb"].data_ptr(), dx.data_ptr(), dx.shape[-1],
                      dh_prev.data_ptr(), am, ls["F"], ls["H"], B, st)
            return
        _lib.call("launch_lstm_bwd_point", dh_heads.data_ptr(), _lib.ptr(dh_rec), _lib.ptr(dc_rec),
                  _lib.ptr(done_t), gates.data_ptr(), c_t.data_ptr(), c_prev.data_ptr(), _lib.ptr(prev_done),
                  dz.data_ptr(), dc_out.data_ptr(), ls["H"], B, st)
        _lib.call("launch_lstm_bwd_gemm", dz.data_ptr(), ls["Kb"].data_ptr(), dx.data_ptr(), dx.shape[-1],
                  dh_prev.data_ptr(), ls["F"], ls["H"], B, st)

    def lstm_wgrad(self, xh, dz, grad_flat, rows_per_chunk: int = 2048):
        ls = self.lstm
        R = xh.numel() // (ls["F"] + ls["H"])
        if ls["x3"]:
            am = ls["amax"]
            _lib.call("launch_lstm_wgrad_x3", xh.data_ptr(), dz.data_ptr(), grad_flat.data_ptr(), ls["k_off"],
                      ls["b_off"], ls["F"], ls["H"], R, rows_per_chunk, am.data_ptr() + 4, am.numel() - 1,
                      am.data_ptr(), _lib.stream())
            return
        _lib.call("launch_lstm_wgrad", xh.data_ptr(), dz.data_ptr(), grad_flat.data_ptr(), ls["k_off"], ls["b_off"],
                  ls["F"], ls["H"], R, rows_per_chunk, _lib.stream())

    def lstm_carry(self, hT, cT, done_last, h0, c0):
        _lib.call("launch_lstm_carry_f32" if self.lstm["x3"] else "launch_lstm_carry", hT.data_ptr(), cT.data_ptr(),
                  done_last.data_ptr(), h0.data_ptr(), c0.data_ptr(), self.lstm["H"], h0.shape[0], _lib.stream())

    # ------------------------------------------------------------------
    def _fwd_ptrs(self, l: int, X, Y, bits, row0: int, p0: int, xrow0: int):
        """Device pointers of a forward launch.  row0 > 0 / p0 > 0 (one path group of the split rollout,
        runtime/engine.py): X, Y and the ReLU bits start at global sample row row0 and the active-module
        tables at path p0, so the kernel sees a population of its own group's paths at t0 = 0 (every kernel
        addresses rows as sample_global(p, s, E, P*E, t0) and bits as [slot][bits_rows] from these bases)."""
        m = self.model
        g = self.geoms[l]
        if row0 == 0 and p0 == 0 and xrow0 == 0:
            return X.data_ptr(), Y.data_ptr(), bits.data_ptr(), m.act_idx.data_ptr(), m.act_cnt.data_ptr()
        xrow = X.shape[-1] * X.element_size()
        yrow = Y.shape[-1] * Y.element_size()
        brow = g.HWo * bits.element_size() if g.kind == "conv" else bits.shape[-1] * bits.element_size()
        i4 = m.act_idx.element_size()
        return (X.data_ptr() + xrow0 * xrow, Y.data_ptr() + row0 * yrow, bits.data_ptr() + row0 * brow,
                m.act_idx.data_ptr() + p0 * self.L * self.M * i4, m.act_cnt.data_ptr() + p0 * self.L * i4)

    @staticmethod
    def _row_ptr(t: torch.Tensor, row: int) -> int:
        """Address of row ``row`` of a [rows, features] buffer (the hi plane of an fp16 pair: lo stays x2_lo away)."""
        return t.data_ptr() + row * t.shape[-1] * t.element_size()

    def _bits_ptr(self, l: int, bits: torch.Tensor, row: int) -> int:
        g = self.geoms[l]
        per_row = g.HWo * bits.element_size() if g.kind == "conv" else bits.shape[-1] * bits.element_size()
        return bits.data_ptr() + row * per_row

    def _tab_ptrs(self, p0: int):
        m = self.model
        i4 = m.act_idx.element_size()
        return m.act_idx.data_ptr() + p0 * self.L * self.M * i4, m.act_cnt.data_ptr() + p0 * self.L * i4

    def prepare_group(self, p0: int, np_: int, rows: int):
        """Allocate path group (p0, np_)'s inverse lists and fc slot planes (outside graph capture)."""
        key = (p0, np_)
        if key not in self._groups:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("path-group buffers first needed inside a graph capture")
            dev = self.model.device
            self._groups[key] = dict(
                inv_path=torch.zeros(self.L, self.M, np_, dtype=torch.int32, device=dev),
                inv_slot=torch.zeros(self.L, self.M, np_, dtype=torch.int32, device=dev),
                inv_cnt=torch.zeros(self.L, self.M, dtype=torch.int32, device=dev),
                ys=torch.empty(8 * self.M * rows * 256, dtype=torch.float32, device=dev))
        return self._groups[key]

    def group_inverse(self, p0: int, np_: int):
        """Rebuild group (p0, np_)'s inverse lists from the population's (csrc/ga.hip inv_group_kernel)."""
        g = self._groups[(p0, np_)]
        _lib.call("launch_inv_group", self.inv_path.data_ptr(), self.inv_slot.data_ptr(), self.inv_cnt.data_ptr(),
                  self.model.P, self.L, self.M, p0, np_, g["inv_path"].data_ptr(), g["inv_slot"].data_ptr(),
                  g["inv_cnt"].data_ptr(), _lib.stream())

    def layer_fwd(self, l: int, X: torch.Tensor, Y: torch.Tensor, bits: torch.Tensor, P: int, E: int, T: int,
                  t0: int, bits_rows: int, row0: int = 0, p0: int = 0, xrow0: Optional[int] = None):
        """Forward of layer l for P paths x E envs x T steps from step t0.  row0/p0/xrow0: a one-step window of
        paths p0..p0+P-1 whose outputs (Y, ReLU bits) start at global sample row row0 and whose inputs start at
        row xrow0 of X (default row0; runtime/engine.py passes the other observation buffer for the bootstrap
        step).  The caller then passes t0 = 0 and T = 1 (see _fwd_ptrs)."""
        g = self.geoms[l]
        m = self.model
        flat = m.store.flat
        out_scale = self.out_scale_last if l == self.L - 1 else 1.0
        st = _lib.stream()
        xrow0 = row0 if xrow0 is None else xrow0
        if (row0 or p0 or xrow0) and (t0 != 0 or T != 1 or p0 + P > m.P or
                                      xrow0 + P * E > X.numel() // X.shape[-1] or
                                      row0 + P * E > Y.numel() // Y.shape[-1]):
            raise ValueError(f"layer {l}: path-group window (row0={row0}, xrow0={xrow0}, p0={p0}, P={P}) out of range")
        xp, yp, bp, aip, acp = self._fwd_ptrs(l, X, Y, bits, row0, p0, xrow0)
        if self.f32:
            _lib.check(Y, torch.float32, name="Y")
            return self._layer_fwd_f32(l, xp, yp, bp, aip, acp, P, E, T, t0, bits_rows, out_scale, st)
        if self.x3:
            return self._layer_fwd_x3(l, X, Y, xp, yp, bp, aip, acp, P, E, T, t0, bits_rows, out_scale, st, p0)
        if g.kind == "conv":
            if (E * g.HWo) % 16 != 0:
                raise ValueError(f"layer {l}: envs_per_path*Ho*Wo must be a multiple of 16")
            f16 = g.u8in and self.Wh0 is not None
            if _lib.USE_FAST and _lib.call_fast(
                    "fast_conv_fwd", xp, int(g.u8in), yp, bp,
                    (self.Wh0 if f16 else self.Wc[l]).data_ptr(), flat.data_ptr(), g.b_off, g.chunk,
                    aip, acp, l, self.L, self.M, g.Hin, g.Win, g.Cin, g.KH, g.KW,
                    g.S, P, E, T, t0, bits_rows, g.in_scale, out_scale, _lib.ptr(self.hcorr0 if f16 else None),
                    self.Wc[l].data_ptr(), st):
                return
            _lib.call("launch_conv_fwd", xp, int(g.u8in), yp, bp,
                      self.Wc[l].data_ptr(), flat.data_ptr(), g.b_off, g.chunk, aip,
                      acp, l, self.L, self.M, g.Hin, g.Win, g.Cin, g.KH, g.KW, g.S, g.Ho, g.Wo,
                      g.K, g.KP, P, E, T, t0, bits_rows, g.in_scale, out_scale, st)
        else:
            _lib.call("launch_fc_fwd", xp, g.ldx, yp, bp, self.Wc[l].data_ptr(),
                      flat.data_ptr(), g.b_off, g.chunk, aip, acp, l, self.L,
                      self.M, g.K, g.KP, g.Cout, P, E, T, t0, bits_rows, out_scale, st)

    def layer_bwd(self, l: int, X: torch.Tensor, G: torch.Tensor, bits: torch.Tensor, grad_flat: torch.Tensor,
                  dX: Optional[torch.Tensor], P: int, E: int, T: int, bits_rows: int, rows_per_chunk: int = 0,
                  part: Optional[str] = None):
        """Backward of layer l.  part (fp32x only): None = both gradients; "d" = the input gradient (plus, on the last
        layer, the G16 amax of the incoming gradient; on fc layers, the masked gradient Gm the weight gradient reads);
        "w" = the weight gradient only, issued after "d" (runtime/engine.py runs it on a side stream)."""
        g = self.geoms[l]
        m = self.model
        flat = m.store.flat
        g_scale = self.out_scale_last if l == self.L - 1 else 1.0
        st = _lib.stream()
        if part is not None and not self.x3:
            raise ValueError("layer_bwd(part=...) is implemented for the fp32x engine")
        if self.f32:
            return self._layer_bwd_f32(l, X, G, bits, grad_flat, dX, P, E, T, bits_rows, g_scale, st)
        if self.x3:
            return self._layer_bwd_x3(l, X, G, bits, grad_flat, dX, P, E, T, bits_rows, g_scale, st, part)
        if self.deterministic:
            return self._layer_bwd_det(l, X, G, bits, grad_flat, dX, P, E, T, bits_rows, g_scale, st)
        if (G.dtype == torch.bfloat16) or (dX is not None and dX.dtype == torch.bfloat16):
            return self._layer_bwd_bf16_grads(l, X, G, bits, grad_flat, dX, P, E, T, bits_rows, g_scale, st)
        if g.kind == "conv":
            fast_w = _lib.USE_FAST and _lib.call_fast(
                "fast_conv_wgrad", X.data_ptr(), int(g.u8in), G.data_ptr(), bits.data_ptr(), grad_flat.data_ptr(),
                g.w_off, g.b_off, g.chunk, m.act_idx.data_ptr(), m.act_cnt.data_ptr(), l, self.L, self.M, g.Hin,
                g.Win, g.Cin, g.KH, g.KW, g.S, P, E, T, bits_rows, g.in_scale, g_scale, st)
            fast_d = dX is None or (_lib.USE_FAST and _lib.call_fast(
                "fast_conv_dgrad", G.data_ptr(), bits.data_ptr(), flat.data_ptr(), g.w_off, g.chunk,
                m.act_idx.data_ptr(), m.act_cnt.data_ptr(), l, self.L, self.M, g.Hin, g.Win, g.Cin, g.KH, g.KW, g.S,
                P, E, T, bits_rows, g_scale, dX.data_ptr(), st))
            if fast_w and fast_d:
                return
        if g.kind == "conv" and not fast_w:
            if rows_per_chunk <= 0:
                rows = T * E * g.HWo
                # ~8 chunks per path keeps >= 8*P workgroups while bounding atomics
                rows_per_chunk = max(32, round_up((rows + 7) // 8, 32))
            _lib.call("launch_conv_wgrad", X.data_ptr(), int(g.u8in), G.data_ptr(), bits.data_ptr(),
                      grad_flat.data_ptr(), g.w_off, g.b_off, g.chunk, m.act_idx.data_ptr(), m.act_cnt.data_ptr(), l,
                      self.L, self.M, g.Hin, g.Win, g.Cin, g.KH, g.KW, g.S, g.Ho, g.Wo, g.K, g.KP, P, E, T,
                      bits_rows, rows_per_chunk, g.in_scale, g_scale, st)
        if g.kind == "conv" and not fast_d:
            if dX is not None:
                _lib.call("launch_conv_dgrad", G.data_ptr(), bits.data_ptr(), flat.data_ptr(), g.w_off, g.chunk,
                          m.act_idx.data_ptr(), m.act_cnt.data_ptr(), l, self.L, self.M, g.Hin, g.Win, g.Cin, g.KH,
                          g.KW, g.S, g.Ho, g.Wo, P, E, T, bits_rows, g_scale, dX.data_ptr(), st)
        if g.kind == "fc":
            # wide fc layers: the dgrad kernel also writes the masked bf16 gradient per active slot,
            # and the weight gradient is a 128 x 256-tile GEMM over it (csrc/trunk_bwd.hip)
            gm = self._gm_buffer(bits_rows) if (dX is not None and g.Cout == 256 and g.K >= self.fc_wgrad_gm_min_k
                                                and self.fc_wgrad_gm) else None
            if dX is not None:
                _lib.call("launch_fc_dgrad", G.data_ptr(), bits.data_ptr(), self.WcT[l].data_ptr(),
                          m.act_idx.data_ptr(), m.act_cnt.data_ptr(), l, self.L, self.M, g.K, g.KP, g.Cout, P, E,
                          T, bits_rows, g_scale, dX.data_ptr(), 0 if gm is None else gm.data_ptr(), st)
            if gm is not None:
                tiles = ((g.K + 127) // 128) * self.M
                nsplit = max(1, min(m.P, -(-512 // tiles)))
                _lib.call("launch_fc_wgrad_gm", X.data_ptr(), g.ldx, gm.data_ptr(), grad_flat.data_ptr(), g.w_off,
                          g.b_off, g.chunk, self.inv_path.data_ptr(), self.inv_slot.data_ptr(),
                          self.inv_cnt.data_ptr(), l, self.M, m.P, g.K, g.Cout, P, E, T, bits_rows, nsplit, st)
            else:
                _lib.call("launch_fc_wgrad", X.data_ptr(), g.ldx, G.data_ptr(), bits.data_ptr(), grad_flat.data_ptr(),
                          g.w_off, g.b_off, g.chunk, self.inv_path.data_ptr(), self.inv_slot.data_ptr(),
                          self.inv_cnt.data_ptr(), l, self.M, m.P, g.K, g.Cout, P, E, T, bits_rows, g_scale, st)

    # reference conv geometries (Hin, Win, Cin, KH, S) of the specialised kernels
    _C1 = (160, 120, 4, 8, 4)
    _C2 = (39, 29, 8, 4, 2)
    _C3 = (18, 13, 8, 3, 1)

    def grad_bf16_layers(self, ring: bool) -> set:
        """Layers l whose output gradient engine.grads[l] is kept in bf16: written by layer l+1's MFMA dgrad and
        read by layer l's slab wgrad (and, for l >= 1, by layer l's MFMA dgrad), all of which round it to bf16
        for their MFMAs anyway (csrc/conv_fast.hip fast_conv_dgrad_bf16 / fast_conv_wgrad_bf16g).  Only those
        reference-geometry kernels take bf16, so every other layer / configuration keeps fp32."""
        if self.f32 or self.x3 or self.deterministic or ring or not _lib.USE_FAST or self.M > 10:
            return set()
        geo = [(g.Hin, g.Win, g.Cin, g.KH, g.S) if g.kind == "conv" else None for g in self.geoms]
        out = set()
        if len(geo) > 1 and geo[0] == self._C1 and self.geoms[0].u8in and geo[1] == self._C2:
            out.add(0)
        if len(geo) > 2 and geo[1] == self._C2 and geo[2] == self._C3:
            out.add(1)
        return out

    # -- fp32x mode (csrc/trunk_x3.hip) -------------------------------------------
    def _x3_lo(self, t: torch.Tensor) -> int:
        return 0 if t.dtype == torch.uint8 else x2_lo(t)

    def _x3_bf16(self, t: torch.Tensor):
        """(pointer, lo offset) of a weight-gradient X operand: an fp16 pair (converted in-kernel), or uint8 frames."""
        if t.dtype == torch.uint8:
            return t.data_ptr(), 0
        return t.data_ptr(), x2_lo(t)

    def _layer_fwd_x3(self, l, X, Y, xp, yp, bp, aip, acp, P, E, T, t0, bits_rows, out_scale, st, p0=0):
        g = self.geoms[l]
        flat = self.model.store.flat
        last = l == self.L - 1
        _lib.check(Y, torch.float32 if last else torch.float16, name="Y")
        ylo = 0 if last else x2_lo(Y)
        wlo = self.Wc[l][0].numel()
        if g.kind == "conv":
            if last:
                raise NotImplementedError("fp32x: a conv layer cannot be the last trunk layer")
            ok = _lib.call_fast("x3_conv_fwd", xp, self._x3_lo(X), int(g.u8in), yp, ylo, bp, self.Wc[l].data_ptr(), wlo,
                                flat.data_ptr(), g.b_off, g.chunk, aip, acp, l, self.L, self.M, g.Hin, g.Win, g.Cin,
                                g.KH, g.KW, g.S, P, E, T, t0, bits_rows, g.in_scale, out_scale, st)
        elif self.fc_fwd_mm and g.Cout == 256 and (g.K >= self.fc_fwd_mm_min_k or P * T * E <= self.fc_fwd_mm_small_rows) \
                and ((P == self.model.P and aip == self.model.act_idx.data_ptr()) or (p0, P) in self._groups):
            # module-major: each module's weight slice read once per 64 rows of the paths using it (a path group:
            # its own inverse lists and slot planes, so two groups' launches never share scratch)
            if P == self.model.P and p0 == 0:
                inv = (self.inv_path, self.inv_slot, self.inv_cnt)
                ys = self._ys_buffer_x3(P * T * E)
            else:
                grp = self._groups[(p0, P)]
                inv = (grp["inv_path"], grp["inv_slot"], grp["inv_cnt"])
                ys = grp["ys"]
                if ys.numel() < 8 * self.M * P * T * E * 256:
                    raise RuntimeError(f"path group ({p0}, {P}): fc slot planes too small for {T * E} rows per path")
            ok = _lib.call_fast("x3_fc_fwd_mm", xp, x2_lo(X), g.ldx, yp, ylo, bp, self.Wc[l].data_ptr(), wlo,
                                flat.data_ptr(), g.b_off, g.chunk, acp, aip, inv[0].data_ptr(),
                                inv[1].data_ptr(), inv[2].data_ptr(), ys.data_ptr(), l, self.L, self.M,
                                g.K, g.KP, g.Cout, P, E, T, t0, bits_rows, out_scale, st)
        else:
            ok = _lib.call_fast("x3_fc_fwd", xp, x2_lo(X), g.ldx, yp, ylo, bp, self.Wc[l].data_ptr(), wlo,
                                flat.data_ptr(), g.b_off, g.chunk, aip, acp, l, self.L, self.M, g.K, g.KP, g.Cout, P, E,
                                T, t0, bits_rows, out_scale, st)
        if not ok:
            raise RuntimeError(f"fp32x: layer {l} forward shape (P={P}, E={E}, T={T}) has no split-bf16 kernel "
                               "(fc layers take <= 32 rows per path and launch)")

    def conv23_fwd(self, l: int, X, Y1, bits1, rows1: int, Y2, bits2, rows2: int, P: int, E: int, T: int,
                   t0: int, row0: int = 0, p0: int = 0) -> bool:
        """fp32x: the forwards of conv layers l (39x29x8 4x4/s2) and l + 1 (18x13x8 3x3/s1) in ONE launch
        (csrc/trunk_x3.hip conv23_fwd_tile_x3, bit-identical to two layer_fwd calls).  False when the pair does not
        have those geometries (the caller then runs layer_fwd twice).  PATHNET_X3_FUSE23=0 disables it."""
        if not self.x3 or not self.fuse23 or l + 1 >= self.L:
            return False
        g1, g2 = self.geoms[l], self.geoms[l + 1]
        if g1.kind != "conv" or g2.kind != "conv" or (g1.Hin, g1.Win, g1.Cin, g1.KH, g1.S, g1.u8in) != self._X3_CONV[1] \
                or (g2.Hin, g2.Win, g2.Cin, g2.KH, g2.S, g2.u8in) != self._X3_CONV[2] or l + 1 == self.L - 1:
            return False
        m = self.model
        for t, nm in ((Y1, "Y1"), (Y2, "Y2")):
            _lib.check(t, torch.float16, name=nm)
        if row0 or p0:
            # one step of path group p0..p0+P-1 (runtime/engine.py split rollout): every operand at the group's
            # first sample row row0, the active-module tables at path p0; the kernel sees P paths at t0 = 0
            if t0 != 0 or T != 1 or p0 + P > m.P or row0 + P * E > min(X.shape[0] * X.shape[1], Y2.shape[0] * Y2.shape[1]):
                raise ValueError(f"conv23_fwd: path-group window (row0={row0}, p0={p0}, P={P}) out of range")
        aip, acp = self._tab_ptrs(p0)
        return _lib.call_fast("x3_conv23_fwd", self._row_ptr(X, row0), x2_lo(X), self._row_ptr(Y1, row0), x2_lo(Y1),
                              self._bits_ptr(l, bits1, row0), rows1, self.Wc[l].data_ptr(), self.Wc[l][0].numel(),
                              g1.b_off, g1.chunk, self._row_ptr(Y2, row0), x2_lo(Y2), self._bits_ptr(l + 1, bits2, row0),
                              rows2, self.Wc[l + 1].data_ptr(), self.Wc[l + 1][0].numel(), g2.b_off, g2.chunk,
                              m.store.flat.data_ptr(), aip, acp, l, self.L, self.M, P, E, T, t0, 1.0, 1.0,
                              _lib.stream())

    def _ys_buffer_x3(self, rows: int) -> torch.Tensor:
        """fp32 module-slot planes [8][M][rows][256] of the module-major fc forward (up to eight k-part planes of
        pre-activations, or one plane of activations; grown before graph capture)."""
        need = 8 * self.M * rows * 256
        if self._ys is None or self._ys.numel() < need:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("fp32x: fc slot buffer first needed inside a graph capture")
            self._ys = torch.empty(need, dtype=torch.float32, device=self.model.device)
        return self._ys

    def _gamax(self, l: int):
        """Device address of layer l's gradient amax (G16), or None below layer 0."""
        return None if l < 0 else self.gamax.data_ptr() + 4 * l

    def _layer_bwd_x3(self, l, X, G, bits, grad_flat, dX, P, E, T, bits_rows, g_scale, st, part=None):
        g = self.geoms[l]
        m = self.model
        flat = m.store.flat
        do_w, do_d = part in (None, "w"), part in (None, "d")
        _lib.check(G, torch.float32, name="G")
        if dX is not None:
            _lib.check(dX, torch.float32, name="dX")
        if l == self.L - 1 and do_d:
            # a backward starts at the last layer: fresh amaxes, the incoming gradient's measured here
            _lib.call("x3_amax_reset", self.gamax.data_ptr(), self.L, st)
            _lib.call("x3_amax", G.data_ptr(), G.numel(), self._gamax(l), st)
        ga, ga_out = self._gamax(l), self._gamax(l - 1)
        xb, xblo = self._x3_bf16(X)
        if g.kind == "conv":
            ok = True
            if do_w:
                ok = _lib.call_fast("x3_conv_wgrad", xb, xblo, int(g.u8in), G.data_ptr(),
                                    bits.data_ptr(), grad_flat.data_ptr(), g.w_off, g.b_off, g.chunk,
                                    m.act_idx.data_ptr(), m.act_cnt.data_ptr(), l, self.L, self.M, g.Hin, g.Win, g.Cin,
                                    g.KH, g.KW, g.S, P, E, T, bits_rows, g.in_scale, g_scale, ga, st)
            if ok and dX is not None and do_d:
                ok = _lib.call_fast("x3_conv_dgrad", G.data_ptr(), bits.data_ptr(), flat.data_ptr(), g.w_off, g.chunk,
                                    m.act_idx.data_ptr(), m.act_cnt.data_ptr(), l, self.L, self.M, g.Hin, g.Win, g.Cin,
                                    g.KH, g.KW, g.S, P, E, T, bits_rows, g_scale, dX.data_ptr(), ga, ga_out, st)
            if not ok:
                raise RuntimeError(f"fp32x: conv layer {l} backward has no split-bf16 kernel")
            return
        # Gm: the masked hi/lo output gradient per active slot -- read by the GEMM input gradient (every fc layer
        # with an input gradient) and by the Gm weight gradient (K >= fc_wgrad_gm_min_k)
        use_gm_wgrad = dX is not None and g.Cout == 256 and g.K >= self.fc_wgrad_gm_min_k and self.fc_wgrad_gm
        gm = self._gm_buffer_x3(bits_rows) if (dX is not None and g.Cout == 256) else None
        gmlo = gm.numel() // 2 if gm is not None else 0
        ok = True
        if dX is not None and do_d:
            ok = _lib.call_fast("x3_fc_dgrad", G.data_ptr(), bits.data_ptr(), self.WcT[l].data_ptr(),
                                self.WcT[l][0].numel(), m.act_idx.data_ptr(), m.act_cnt.data_ptr(), l, self.L, self.M,
                                g.K, g.KP, g.Cout, P, E, T, bits_rows, g_scale, dX.data_ptr(), _lib.ptr(gm), gmlo, ga,
                                ga_out, st)
        if not do_w:
            pass
        elif ok and use_gm_wgrad:
            tiles = ((g.K + 127) // 128) * self.M
            # workgroups ~ a whole number of rounds of one per CU (fc_wgrad_gm_x3 holds 102 KB of LDS): 110 tiles x 7
            # = 770 = 3.0 rounds on 256 CUs, where 110 x 5 = 550 left the third round 15 % full
            wgs = self.fc_wgrad_gm_wgs if m.P > 16 else self.fc_wgrad_gm_wgs_small
            nsplit = max(1, min(m.P, -(-wgs // tiles)))
            ok = _lib.call_fast("x3_fc_wgrad_gm", xb, xblo, g.ldx, gm.data_ptr(), gmlo,
                                grad_flat.data_ptr(), g.w_off, g.b_off, g.chunk, self.inv_path.data_ptr(),
                                self.inv_slot.data_ptr(), self.inv_cnt.data_ptr(), l, self.M, m.P, g.K, g.Cout, P, E, T,
                                bits_rows, nsplit, ga, st)
        elif ok:
            ok = _lib.call_fast("x3_fc_wgrad", xb, xblo, g.ldx, G.data_ptr(), bits.data_ptr(),
                                grad_flat.data_ptr(), g.w_off, g.b_off, g.chunk, self.inv_path.data_ptr(),
                                self.inv_slot.data_ptr(), self.inv_cnt.data_ptr(), l, self.M, m.P, g.K, g.Cout, P, E, T,
                                bits_rows, g_scale, ga, st)
        if not ok:
            raise RuntimeError(f"fp32x: fc layer {l} backward has no split-bf16 kernel")

    def _gm_buffer_x3(self, bits_rows: int) -> torch.Tensor:
        """[2][M][bits_rows][256] 16-bit hi/lo scratch for the masked fc gradient: fp16 pair of G * 2^e (G16; a bf16
        tensor only as storage), allocated before graph capture."""
        n = 2 * self.M * bits_rows * 256
        buf = getattr(self, "_gm", None)
        if buf is None or buf.numel() != n:
            buf = torch.empty(n, dtype=torch.bfloat16, device=self.model.store.flat.device)
            self._gm = buf
        return buf

    # -- fp32 mode (csrc/trunk_f32.hip) ------------------------------------------
    def _layer_fwd_f32(self, l, xp, yp, bp, aip, acp, P, E, T, t0, bits_rows, out_scale, st):
        g = self.geoms[l]
        flat = self.model.store.flat
        if g.kind == "conv":
            if (E * g.HWo) % 16 != 0:
                raise ValueError(f"layer {l}: envs_per_path*Ho*Wo must be a multiple of 16")
            _lib.call("launch_conv_fwd_f32", xp, int(g.u8in), yp, bp,
                      self.Wc[l].data_ptr(), flat.data_ptr(), g.b_off, g.chunk, aip,
                      acp, l, self.L, self.M, g.Hin, g.Win, g.Cin, g.KH, g.KW, g.S, g.Ho, g.Wo,
                      g.K, g.KP, P, E, T, t0, bits_rows, g.in_scale, out_scale, st)
        else:
            _lib.call("launch_fc_fwd_f32", xp, g.ldx, yp, bp, self.Wc[l].data_ptr(),
                      flat.data_ptr(), g.b_off, g.chunk, aip, acp, l, self.L,
                      self.M, g.K, g.KP, g.Cout, P, E, T, t0, bits_rows, out_scale, st)

    def wgrad_chunks(self, l: int, P: int, E: int, T: int) -> int:
        """Row chunks per path of the fp32 conv wgrad (>= ~1024 workgroups), matching the launcher's rounding."""
        g = self.geoms[l]
        rows = T * E * g.HWo
        want = max(1, min(-(-rows // 32), -(-1024 // P)))
        rpc = round_up(-(-rows // want), 32)
        return -(-rows // rpc)

    def _part_buffer(self, numel: int) -> torch.Tensor:
        if self._part is None or self._part.numel() < numel:
            self._part = torch.empty(numel, dtype=torch.float32, device=self.model.store.flat.device)
        return self._part

    def _layer_bwd_bf16_grads(self, l, X, G, bits, grad_flat, dX, P, E, T, bits_rows, g_scale, st):
        """Conv layer with a bf16 output gradient G and/or a bf16 input gradient dX (grad_bf16_layers): no
        fallback kernel reads or writes those, so an unspecialised shape raises."""
        g = self.geoms[l]
        m = self.model
        flat = m.store.flat
        if g.kind != "conv":
            raise RuntimeError(f"layer {l}: bf16 activation gradients are for the conv layers")
        args = (g.w_off, g.b_off, g.chunk, m.act_idx.data_ptr(), m.act_cnt.data_ptr(), l, self.L, self.M, g.Hin,
                g.Win, g.Cin, g.KH, g.KW, g.S, P, E, T, bits_rows, g.in_scale, g_scale, st)
        g_bf = G.dtype == torch.bfloat16
        ok = _lib.call_fast("fast_conv_wgrad_bf16g" if g_bf else "fast_conv_wgrad", X.data_ptr(), int(g.u8in),
                            G.data_ptr(), bits.data_ptr(), grad_flat.data_ptr(), *args)
        if ok and dX is not None:
            ok = _lib.call_fast("fast_conv_dgrad_bf16", G.data_ptr(), int(g_bf), bits.data_ptr(), flat.data_ptr(),
                                g.w_off, g.chunk, m.act_idx.data_ptr(), m.act_cnt.data_ptr(), l, self.L, self.M, g.Hin,
                                g.Win, g.Cin, g.KH, g.KW, g.S, P, E, T, bits_rows, g_scale, dX.data_ptr(),
                                int(dX.dtype == torch.bfloat16), st)
        if not ok:
            raise RuntimeError(f"layer {l}: bf16 activation gradients need the specialised kernels "
                               "(HipPathNet.grad_bf16_layers)")

    def _conv_wgrad_ordered(self, l, X, G, bits, grad_flat, P, E, T, bits_rows, g_scale, st):
        """Conv weight gradient with fixed-order reductions (uint8 / bf16 / fp32 input, fp32 MFMA)."""
        g = self.geoms[l]
        m = self.model
        if G.dtype != torch.float32:
            raise TypeError("the ordered conv wgrad takes an fp32 output gradient")
        nch = self.wgrad_chunks(l, P, E, T)
        part = self._part_buffer(P * nch * self.M * (g.K * 8 + 8))
        xkind = 0 if g.u8in else (2 if X.dtype == torch.float32 else 1)
        _lib.call("launch_conv_wgrad_f32", X.data_ptr(), xkind, G.data_ptr(), bits.data_ptr(),
                  grad_flat.data_ptr(), part.data_ptr(), g.w_off, g.b_off, g.chunk, m.act_idx.data_ptr(),
                  m.act_cnt.data_ptr(), self.inv_path.data_ptr(), self.inv_slot.data_ptr(),
                  self.inv_cnt.data_ptr(), l, self.L, self.M, m.P, g.Hin, g.Win, g.Cin, g.KH, g.KW, g.S, g.Ho,
                  g.Wo, g.K, g.KP, P, E, T, bits_rows, nch, g.in_scale, g_scale, st)

    def _fc_wgrad_ordered(self, l, X, G, bits, grad_flat, P, E, T, bits_rows, g_scale, st):
        g = self.geoms[l]
        m = self.model
        _lib.call("launch_fc_wgrad_f32", X.data_ptr(), 2 if X.dtype == torch.float32 else 1, g.ldx, G.data_ptr(),
                  bits.data_ptr(), grad_flat.data_ptr(), g.w_off, g.b_off, g.chunk, self.inv_path.data_ptr(),
                  self.inv_slot.data_ptr(), self.inv_cnt.data_ptr(), l, self.M, m.P, g.K, g.Cout, P, E, T, bits_rows,
                  g_scale, st)

    def _layer_bwd_det(self, l, X, G, bits, grad_flat, dX, P, E, T, bits_rows, g_scale, st):
        """bf16 engine, deterministic mode: the bf16 dgrad kernels (no atomics) + ordered fp32 weight gradients."""
        g = self.geoms[l]
        m = self.model
        flat = m.store.flat
        if g.kind == "conv":
            self._conv_wgrad_ordered(l, X, G, bits, grad_flat, P, E, T, bits_rows, g_scale, st)
            if dX is not None and not (_lib.USE_FAST and _lib.call_fast(
                    "fast_conv_dgrad", G.data_ptr(), bits.data_ptr(), flat.data_ptr(), g.w_off, g.chunk,
                    m.act_idx.data_ptr(), m.act_cnt.data_ptr(), l, self.L, self.M, g.Hin, g.Win, g.Cin, g.KH, g.KW,
                    g.S, P, E, T, bits_rows, g_scale, dX.data_ptr(), st)):
                _lib.call("launch_conv_dgrad", G.data_ptr(), bits.data_ptr(), flat.data_ptr(), g.w_off, g.chunk,
                          m.act_idx.data_ptr(), m.act_cnt.data_ptr(), l, self.L, self.M, g.Hin, g.Win, g.Cin, g.KH,
                          g.KW, g.S, g.Ho, g.Wo, P, E, T, bits_rows, g_scale, dX.data_ptr(), st)
            return
        if dX is not None:
            _lib.call("launch_fc_dgrad", G.data_ptr(), bits.data_ptr(), self.WcT[l].data_ptr(),
                      m.act_idx.data_ptr(), m.act_cnt.data_ptr(), l, self.L, self.M, g.K, g.KP, g.Cout, P, E,
                      T, bits_rows, g_scale, dX.data_ptr(), None, st)
        self._fc_wgrad_ordered(l, X, G, bits, grad_flat, P, E, T, bits_rows, g_scale, st)

    def _layer_bwd_f32(self, l, X, G, bits, grad_flat, dX, P, E, T, bits_rows, g_scale, st):
        g = self.geoms[l]
        m = self.model
        flat = m.store.flat
        if g.kind == "conv":
            self._conv_wgrad_ordered(l, X, G, bits, grad_flat, P, E, T, bits_rows, g_scale, st)
            if dX is not None:
                _lib.call("launch_conv_dgrad_f32", G.data_ptr(), bits.data_ptr(), flat.data_ptr(), g.w_off, g.chunk,
                          m.act_idx.data_ptr(), m.act_cnt.data_ptr(), l, self.L, self.M, g.Hin, g.Win, g.Cin, g.KH,
                          g.KW, g.S, g.Ho, g.Wo, P, E, T, bits_rows, g_scale, dX.data_ptr(), st)
            return
        if dX is not None:
            _lib.call("launch_fc_dgrad_f32", G.data_ptr(), bits.data_ptr(), self.WcT[l].data_ptr(),
                      m.act_idx.data_ptr(), m.act_cnt.data_ptr(), l, self.L, self.M, g.K, g.KP, g.Cout, P, E, T,
                      bits_rows, g_scale, dX.data_ptr(), st)
        self._fc_wgrad_ordered(l, X, G, bits, grad_flat, P, E, T, bits_rows, g_scale, st)

    def _gm_buffer(self, bits_rows: int) -> torch.Tensor:
        """[M][bits_rows][256] bf16 scratch for the masked fc gradient (allocated before graph capture)."""
        n = self.M * bits_rows * 256
        buf = getattr(self, "_gm", None)
        if buf is None or buf.numel() < n:
            buf = torch.empty(n, dtype=torch.bfloat16, device=self.model.store.flat.device)
            self._gm = buf
        return buf

    # -- first layer on the frame ring (frames [B][T+4][H*W] u8, fc [T+1][B] u8) --------
    def _check_ring(self, frames, fc, P, E, steps):
        g = self.geoms[0]
        _lib.check(frames, torch.uint8, name="frames")
        _lib.check(fc, torch.uint8, name="fc")
        if frames.dim() != 3 or frames.shape[0] != P * E or frames.shape[2] != g.Hin * g.Win:
            raise ValueError(f"frames shape {tuple(frames.shape)} != [P*E, slots, {g.Hin * g.Win}]")
        if frames.shape[1] < steps + 3 or fc.numel() < steps * P * E:
            raise ValueError("frame ring too short for the requested steps")

    def ring_fwd(self, frames, fc, Y, bits, P: int, E: int, T: int, t0: int, bits_rows: int, p0: int = 0,
                 np_: Optional[int] = None, rbase: int = 0):
        """First layer on the frame ring, P paths x E envs x T steps from t0.  p0/np_ (fp32x): paths p0..p0+np_-1 of
        step t0 only (one group of the split rollout): frames, fc, Y, bits and the module tables are passed at the
        group's base (frames at env p0*E, slot t0; fc and the output rows at row t0*P*E + p0*E), so the kernel
        sees np_ paths at t0 = 0."""
        self._check_ring(frames, fc, P, E, t0 + T)
        g = self.geoms[0]
        m = self.model
        out_scale = self.out_scale_last if self.L == 1 else 1.0
        grouped = np_ is not None and (p0, np_) != (0, P)
        if grouped and (not self.x3 or T != 1 or p0 < 0 or np_ <= 0 or p0 + np_ > P):
            raise ValueError(f"ring_fwd: path group (p0={p0}, np={np_}) needs fp32x, T = 1 and paths within {P}")
        if self.x3:
            _lib.check(Y, torch.float16, name="Y")
            if grouped:
                B = P * E
                row0 = t0 * B + p0 * E
                fp = frames.data_ptr() + (p0 * E * frames.shape[1] + t0) * frames.shape[2]
                aip, acp = self._tab_ptrs(p0)
                args = (fp, fc.data_ptr() + row0, self._row_ptr(Y, row0), x2_lo(Y), self._bits_ptr(0, bits, row0),
                        aip, acp, np_, 0)
            else:
                args = (frames.data_ptr(), fc.data_ptr(), Y.data_ptr(), x2_lo(Y), bits.data_ptr(),
                        m.act_idx.data_ptr(), m.act_cnt.data_ptr(), P, t0)
            fp, fcp, yp, ylo, bp, aip, acp, Pk, t0k = args
            if grouped and rbase:
                raise ValueError("ring_fwd: a path group of the split rollout needs the unwrapped ring (rbase 0)")
            ok = _lib.call_fast("x3_conv1_ring_fwd", fp, fcp, yp, ylo, bp, self.Wc[0].data_ptr(), self.Wc[0][0].numel(),
                                m.store.flat.data_ptr(), g.b_off, g.chunk, aip, acp, self.L, self.M, Pk, E, T, t0k,
                                frames.shape[1], rbase, bits_rows, g.in_scale, out_scale, _lib.stream())
            if not ok:
                raise RuntimeError(f"fp32x: frame-ring forward has no kernel for P={P}, E={E}, M={self.M}")
            return
        if rbase:
            raise ValueError("ring_fwd: the bf16 ring kernels read the unwrapped ring (rbase 0)")
        _lib.call("fast_conv1_ring_fwd", frames.data_ptr(), fc.data_ptr(), Y.data_ptr(), bits.data_ptr(),
                  self.Wh_ring.data_ptr(), m.store.flat.data_ptr(), g.b_off, g.chunk, m.act_idx.data_ptr(),
                  m.act_cnt.data_ptr(), 0, self.L, self.M, P, E, T, t0, frames.shape[1], bits_rows, g.in_scale,
                  out_scale, self.hcorr0.data_ptr(), self.Wc_ring.data_ptr(), _lib.stream())

    def ring_wgrad(self, frames, fc, G, bits, grad_flat, P: int, E: int, T: int, bits_rows: int, rbase: int = 0):
        self._check_ring(frames, fc, P, E, T)
        g = self.geoms[0]
        m = self.model
        g_scale = self.out_scale_last if self.L == 1 else 1.0
        if self.x3:
            _lib.check(G, torch.float32, name="G")
            ok = _lib.call_fast("x3_conv1_ring_wgrad", frames.data_ptr(), fc.data_ptr(), G.data_ptr(), bits.data_ptr(),
                                grad_flat.data_ptr(), g.w_off, g.b_off, g.chunk, m.act_idx.data_ptr(),
                                m.act_cnt.data_ptr(), self.L, self.M, P, E, T, frames.shape[1], rbase, bits_rows,
                                g.in_scale, g_scale, self._gamax(0), _lib.stream())
            if not ok:
                raise RuntimeError(f"fp32x: frame-ring weight gradient has no kernel for P={P}, E={E}, M={self.M}")
            return
        if rbase:
            raise ValueError("ring_wgrad: the bf16 ring kernels read the unwrapped ring (rbase 0)")
        _lib.call("fast_conv1_ring_wgrad", frames.data_ptr(), fc.data_ptr(), G.data_ptr(), bits.data_ptr(),
                  grad_flat.data_ptr(), g.w_off, g.b_off, g.chunk, m.act_idx.data_ptr(), m.act_cnt.data_ptr(), 0,
                  self.L, self.M, P, E, T, frames.shape[1], bits_rows, g.in_scale, g_scale, _lib.stream())

    # ------------------------------------------------------------------
    def alloc_bits(self, l: int, steps: int, B: int):
        g = self.geoms[l]
        dev = self.model.device
        if g.kind == "conv":
            rows = steps * B * g.HWo
            return torch.zeros(self.M, rows, dtype=torch.uint8, device=dev), rows
        rows = steps * B
        return torch.zeros(self.M, rows, g.Cout // 16, dtype=torch.int16, device=dev), rows

    def fc_heads_fwd(self, X, Y, bits, bits_rows: int, logits, value, actions, seed, ctr, t: int, T: int, P: int,
                     E: int, t0: int, greedy=False, task=0, row_base=0) -> bool:
        """fp32x: the last trunk layer (an fc layer of 256 outputs over 256 inputs) AND the heads + sampling of one
        rollout step in one launch (csrc/trunk_x3.hip fc_heads_fwd_x3: bit-identical to layer_fwd + heads_fwd).
        X / Y / bits: the layer's full [steps, B, ...] buffers (step t0's rows are used); logits / value / actions:
        step t's [B] rows.  False when the shape is not covered (the caller then runs the two launches);
        PATHNET_X3_FUSE_HEADS=0 disables it."""
        l = self.L - 1
        g = self.geoms[l]
        m = self.model
        if not (self.x3 and self.fuse_heads and g.kind == "fc" and self.lstm is None and l > 0):
            return False
        h = m.store.layout.heads[task if m.cfg.per_task_heads else 0]
        _lib.check(Y, torch.float32, name="Y")
        B = P * E
        if X.shape[-2] != B or Y.shape[-2] != B or logits.numel() < B * m.cfg.num_actions or value.numel() < B \
                or actions.numel() < B:
            raise ValueError("fc_heads_fwd: buffers do not hold one step of P*E samples")
        return _lib.call_fast("x3_fc_heads_fwd", X.data_ptr(), x2_lo(X), g.ldx, Y.data_ptr(), bits.data_ptr(),
                              self.Wc[l].data_ptr(), self.Wc[l][0].numel(), m.store.flat.data_ptr(), g.b_off, g.chunk,
                              m.act_idx.data_ptr(), m.act_cnt.data_ptr(), l, self.L, self.M, g.K, g.KP, g.Cout, P, E,
                              t0, bits_rows, self.out_scale_last, h["pw"], h["pb"], h["vw"], h["vb"],
                              m.cfg.num_actions, logits.data_ptr(), value.data_ptr(), actions.data_ptr(),
                              seed & 0xFFFFFFFF, ctr.data_ptr(), t, T, int(greedy), int(row_base) & 0xFFFFFFFF,
                              _lib.stream())

    def heads_fwd(self, feat, logits, value, actions, seed, ctr, t, T, greedy=False, task=0, b0=0, b1=None,
                  row_base=0):
        """Heads + Gumbel-max sampling of samples [b0, b1) of feat [B, F] (default all; the split rollout
        passes one path group's rows, runtime/engine.py).  Sample b draws the RNG of global sample row_base + b
        (row_base = the rank's first env of the population: sharding-invariant sampling)."""
        m = self.model
        h = m.store.layout.heads[task if m.cfg.per_task_heads else 0]
        B = feat.shape[0] if b1 is None else b1
        F = feat.shape[1]
        A = m.cfg.num_actions
        _lib.check(feat, self.feat_dtype, name="feat")
        if not 0 <= b0 < B <= feat.shape[0]:
            raise ValueError(f"heads_fwd: sample range [{b0}, {B}) outside [0, {feat.shape[0]})")
        _lib.call("launch_heads_fwd_sample_f32" if self.feat_dtype == torch.float32 else "launch_heads_fwd_sample",
                  feat.data_ptr(), F,
                  m.store.flat.data_ptr(), h["pw"], h["pb"], h["vw"], h["vb"], A, B, logits.data_ptr(),
                  value.data_ptr(), actions.data_ptr(), seed & 0xFFFFFFFF, ctr.data_ptr(), t, T, int(greedy), b0,
                  int(row_base) & 0xFFFFFFFF, _lib.stream())

    def heads_bwd(self, feat, dlogits, dvalue, grad_flat, dfeat, task=0):
        m = self.model
        h = m.store.layout.heads[task if m.cfg.per_task_heads else 0]
        N, F = feat.shape
        _lib.check(feat, self.feat_dtype, name="feat")
        A = m.cfg.num_actions
        if self.deterministic:
            n = _lib.lib().heads_bwd_part_numel(N, F, A)
            if self._hpart is None or self._hpart.numel() < n:
                self._hpart = torch.empty(n, dtype=torch.float32, device=feat.device)
            _lib.call("launch_heads_bwd_det", feat.data_ptr(), int(self.f32), F, dlogits.data_ptr(),
                      dvalue.data_ptr(), N, A, m.store.flat.data_ptr(), h["pw"], h["pb"], h["vw"], h["vb"],
                      grad_flat.data_ptr(), dfeat.data_ptr(), self._hpart.data_ptr(), _lib.stream())
            return
        # partials buffer of the 32-row split (csrc/heads.hip launch_heads_bwd_split; the 128-row atomic kernel
        # unless heads_set_bwd_rows(32)); grown outside graph capture like _hpart
        n = _lib.lib().heads_bwd_split_numel(N, F, A)
        if self._hsplit is None or self._hsplit.numel() < n:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("heads backward partials first needed inside a graph capture")
            self._hsplit = torch.empty(n, dtype=torch.float32, device=feat.device)
        _lib.call("launch_heads_bwd_split", feat.data_ptr(), int(self.feat_dtype == torch.float32), F,
                  dlogits.data_ptr(), dvalue.data_ptr(), N, A, m.store.flat.data_ptr(), h["pw"], h["pb"], h["vw"],
                  h["vb"], grad_flat.data_ptr(), dfeat.data_ptr(), self._hsplit.data_ptr(), _lib.stream())

    # -- standalone forward (tests / acting): obs [B, ...] -> feat [B, F] --------
    def trunk(self, obs: torch.Tensor, samples_per_path: int):
        m = self.model
        P, E = m.P, samples_per_path
        B = P * E
        x = self._prep_input(obs)
        out = None
        for l, g in enumerate(self.geoms):
            Y = self.alloc_act(l, (B, g.out_feat))
            bits, rows = self.alloc_bits(l, 1, B)
            self.layer_fwd(l, x, Y, bits, P, E, 1, 0, rows)
            x = Y
            out = Y
        return out.float()

    def _prep_input(self, obs):
        if self.pixels:
            return _lib.check(obs.contiguous(), torch.uint8, name="obs")
        if self.f32:
            return obs.float().reshape(obs.shape[0], -1).contiguous()
        if obs.dtype == torch.bfloat16 and obs.shape[-1] == 8:
            return obs.contiguous()
        from .envs import obs_to_bf16_padded
        return obs_to_bf16_padded(obs.float())

    def heads(self, feat, task=0):
        from ..models.pathnet import heads_ref
        return heads_ref(self.model.store, feat, task)
