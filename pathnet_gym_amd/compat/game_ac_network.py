"""``GameACPathNetNetwork`` / ``GameACPathNetLSTMNetwork`` with the reference API.

Reference: ``game_ac_network.py:11-85`` (base: loss, sync), ``:113-271`` (FF),
``:303-521`` (LSTM).  One instance = one agent (one genotype, batch 1 at act
time), as in the reference's per-worker graphs.  Weights live in a
``ParamStore`` flat buffer; instances created with the same
``thread_index`` share it (the reference shares TF scope ``net_<thread_index>``
-- always ``net_0`` -- on the parameter server).

``sess`` arguments are accepted and ignored: ``run_policy_and_value(sess, s)``
and ``run_policy_and_value(s)`` both work.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from ..config import ACTION_SIZEZ, PathNetConfig, reference_pixel_layers
from ..models.acnet import ACPathNet
from ..models.pathnet import ParamStore, Segment

_SHARED: Dict[Tuple, ParamStore] = {}


def _flag(FLAGS, name, default):
    return getattr(FLAGS, name, default) if FLAGS not in (None, "") else default


def config_from_flags(FLAGS=None, use_lstm: bool = False) -> PathNetConfig:
    """Reference flags (--L --M --N --kernel_num --stride_size) -> PathNetConfig."""
    L = int(_flag(FLAGS, "L", 4))
    kernels = [int(k) for k in str(_flag(FLAGS, "kernel_num", "8,4,3")).split(",")]
    strides = [int(s) for s in str(_flag(FLAGS, "stride_size", "4,2,1")).split(",")]
    return PathNetConfig(L=L, M=int(_flag(FLAGS, "M", 10)), N=int(_flag(FLAGS, "N", 4)),
                         layers=reference_pixel_layers(L, kernels, strides),
                         trunk_scale="none" if use_lstm else "M", use_lstm=use_lstm,
                         num_actions=max(ACTION_SIZEZ))


def _arg(a, b):
    """(sess, x) or (x,) call styles."""
    return a if b is None else b


class GameACPathNetNetwork:
    use_lstm = False

    def __init__(self, training_stage: int, thread_index: int, device="cpu", FLAGS=None,
                 store: Optional[ParamStore] = None, seed: int = 1):
        self.training_stage = training_stage
        self._action_size = ACTION_SIZEZ[training_stage]
        self._thread_index = thread_index
        self._device = torch.device("cpu" if str(device).startswith("/cpu") else device)
        self.task_index = int(_flag(FLAGS, "task_index", 0) or 0)
        self.cfg = config_from_flags(FLAGS, self.use_lstm)
        self.model = ACPathNet(self.cfg, 1, self._device, "torch", seed=seed)
        if store is None:
            key = (thread_index, str(self._device), self.cfg.L, self.cfg.M, self.use_lstm)
            store = _SHARED.setdefault(key, self.model.store)
        self.model.store = store
        L, M = self.cfg.L, self.cfg.M
        self.geopath = np.ones((L, M), np.float32)           # geopath_initializer: all 1.0 (pathnet.py:25-30)
        self.fixed_path = np.zeros((L, M), np.float32)
        self.model.set_paths(self.geopath[None])
        self.entropy_beta = 0.01
        self.lstm_state_out = None
        self.reset_state()

    # -- weights / genotype ---------------------------------------------------
    @property
    def store(self) -> ParamStore:
        return self.model.store

    def set_geopath(self, g):
        self.geopath = np.asarray(g, np.float32).copy()
        self.model.set_paths(self.geopath[None])

    def get_geopath(self, sess=None) -> np.ndarray:
        return self.geopath.astype(float).copy()

    def set_fixed_path(self, fixed_path):
        self.fixed_path = np.asarray(fixed_path, np.float32).copy()

    def set_training_stage(self, training_stage: int):
        self.training_stage = training_stage
        self._action_size = ACTION_SIZEZ[training_stage]

    def _ordered_segments(self) -> List[Tuple[Segment, bool]]:
        """Reference variable order with trainability: trunk (W,b per module), policy, value, [lstm]."""
        segs = self.store.layout.segments
        trunk = [s for s in segs if s.layer >= 0]
        heads = [s for s in segs if s.name.startswith(("policy", "value"))]
        lstm = [s for s in segs if s.name.startswith("lstm")]
        out = [(s, self.fixed_path[s.layer, s.module] == 0.0) for s in trunk]
        return out + [(s, True) for s in heads + lstm]

    def _view(self, s: Segment) -> torch.Tensor:
        return self.store.flat.detach()[s.offset:s.offset + s.numel].view(s.shape)

    def get_vars(self) -> List[torch.Tensor]:
        """Non-frozen variables in reference order (game_ac_network.py:239-253 / :493-507)."""
        return [self._view(s) for s, tr in self._ordered_segments() if tr]

    def get_vars_idx(self) -> List[int]:
        """0/1 per variable of the FULL list (game_ac_network.py:255-271 / :509-521)."""
        return [int(tr) for _, tr in self._ordered_segments()]

    def all_vars(self) -> List[torch.Tensor]:
        return [self._view(s) for s, _ in self._ordered_segments()]

    def grads_for(self, flat_grad: torch.Tensor, full: bool = True) -> List[torch.Tensor]:
        """Slice a flat gradient into per-variable gradients aligned with all_vars()/get_vars()."""
        return [flat_grad[s.offset:s.offset + s.numel].view(s.shape)
                for s, tr in self._ordered_segments() if full or tr]

    def sync_from(self, src_network, name=None):
        """Copy every variable from ``src_network`` (game_ac_network.py:73-85)."""
        with torch.no_grad():
            self.store.flat.copy_(src_network.store.flat.to(self.store.flat.device))

    # -- loss (game_ac_network.py:20-59) ---------------------------------------
    def prepare_loss(self, entropy_beta: float):
        self.entropy_beta = float(entropy_beta)

    def loss(self, s, a, td, r, initial_lstm_state=None) -> torch.Tensor:
        """total_loss for a rollout: s [T,H,W,C], a one-hot [T,A], td [T], r [T] (sums over T)."""
        pi, v = self._forward(s, initial_lstm_state, grad=True)
        a = torch.as_tensor(np.asarray(a), dtype=torch.float32, device=self._device)
        td = torch.as_tensor(np.asarray(td), dtype=torch.float32, device=self._device)
        r = torch.as_tensor(np.asarray(r), dtype=torch.float32, device=self._device)
        log_pi = torch.log(pi.clamp(1e-20, 1.0))
        entropy = -(pi * log_pi).sum(1)
        policy_loss = -((log_pi * a).sum(1) * td + entropy * self.entropy_beta).sum()
        value_loss = 0.5 * 0.5 * ((r - v) ** 2).sum()          # 0.5 * tf.nn.l2_loss
        return policy_loss + value_loss

    # -- forward ------------------------------------------------------------------
    def _batch(self, s) -> torch.Tensor:
        x = torch.as_tensor(np.asarray(s), dtype=torch.float32, device=self._device)
        if x.dim() == len(self.cfg.input_shape):
            x = x[None]
        return x

    def _forward(self, s, state=None, grad=False):
        x = self._batch(s)
        with torch.set_grad_enabled(grad):
            feat = self.model.trunk(x, x.shape[0])
            if self.use_lstm:
                k, b = self.store.lstm()
                h, c = state if state is not None else self.lstm_state_out
                h = torch.as_tensor(np.asarray(h), dtype=torch.float32, device=self._device).reshape(1, -1)
                c = torch.as_tensor(np.asarray(c), dtype=torch.float32, device=self._device).reshape(1, -1)
                from ..models.pathnet import lstm_cell_ref
                outs = []
                for t in range(feat.shape[0]):           # dynamic_rnn over the rollout (:411-416)
                    h, c = lstm_cell_ref(feat[t:t + 1], h, c, k, b)
                    outs.append(h)
                feat = torch.cat(outs)
                self._last_state = (h.detach().cpu().numpy(), c.detach().cpu().numpy())
            from ..models.pathnet import heads_ref
            logits, v = heads_ref(self.store, feat, self.training_stage)
        return F.softmax(logits, -1), v

    def run_policy_and_value(self, sess, s_t=None):
        pi, v = self._forward(_arg(sess, s_t))
        if self.use_lstm:
            self.lstm_state_out = self._last_state
        return pi[0].cpu().numpy(), float(v[0])

    def run_policy(self, sess, s_t=None):
        pi, _ = self._forward(_arg(sess, s_t))
        if self.use_lstm:
            self.lstm_state_out = self._last_state
        return pi[0].cpu().numpy()

    def run_value(self, sess, s_t=None):
        _, v = self._forward(_arg(sess, s_t))      # LSTM state rolled back (:467-481): not stored
        return float(v[0])

    def reset_state(self):
        if self.use_lstm:
            H = self.cfg.lstm_size
            self.lstm_state_out = (np.zeros((1, H), np.float32), np.zeros((1, H), np.float32))


class GameACPathNetLSTMNetwork(GameACPathNetNetwork):
    use_lstm = True
