"""``RMSPropApplier`` with the reference call shape (``rmsprop_applier.py:9-106``).

Per-variable slots ``rms`` (initialised to 1.0) and ``momentum`` (zeros);
``apply_gradients(var_list, grad_list)`` clips each gradient by its own L2
norm (``clip_by_norm(g, clip_norm)``, :104) and applies TF ``ApplyRMSProp``
(epsilon inside the sqrt, :82-89) in place.  Variables are tensors (e.g. the
flat-buffer views returned by ``GameACPathNetNetwork.get_vars()``), so an
update writes straight into the shared super-network.

The learning rate is a float, or anything callable returning one (the
reference feeds a placeholder); ``apply_gradients(..., learning_rate=x)``
overrides it per call.  The population engine uses the fused
multi-tensor version of the same math (``algo/optim.py``, ``csrc/optim.hip``).
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import torch


class RMSPropApplier:
    def __init__(self, learning_rate, decay: float = 0.9, momentum: float = 0.0, epsilon: float = 1e-10,
                 clip_norm: float = 40.0, device="/cpu:0", name: str = "RMSPropApplier"):
        self._name = name
        self._learning_rate = learning_rate
        self._decay = decay
        self._momentum = momentum
        self._epsilon = epsilon
        self._clip_norm = clip_norm
        self._device = device
        self._slots: Dict[str, Dict[int, torch.Tensor]] = {"rms": {}, "momentum": {}}

    # -- slots (rmsprop_applier.py:34-73) -------------------------------------
    @staticmethod
    def _key(var: torch.Tensor):
        return (var.data_ptr(), tuple(var.shape))

    def _create_slots(self, var_list: Sequence[torch.Tensor]):
        for v in var_list:
            k = self._key(v)
            if k not in self._slots["rms"]:
                self._slots["rms"][k] = torch.ones_like(v, dtype=torch.float32)
                self._slots["momentum"][k] = torch.zeros_like(v, dtype=torch.float32)

    def get_slot(self, var: torch.Tensor, name: str) -> torch.Tensor:
        return self._slots[name][self._key(var)]

    def _lr(self, override=None) -> float:
        lr = self._learning_rate if override is None else override
        return float(lr() if callable(lr) else lr)

    # -- apply (rmsprop_applier.py:79-106) -------------------------------------
    @torch.no_grad()
    def _apply_dense(self, grad: torch.Tensor, var: torch.Tensor, lr: float):
        ms = self.get_slot(var, "rms")
        mom = self.get_slot(var, "momentum")
        g = grad.to(var.device, torch.float32)
        ms.mul_(self._decay).addcmul_(g, g, value=1.0 - self._decay)
        mom.mul_(self._momentum).add_(lr * g / torch.sqrt(ms + self._epsilon))
        var.sub_(mom.to(var.dtype))

    @torch.no_grad()
    def apply_gradients(self, var_list: Sequence[torch.Tensor], accum_grad_list: Sequence[torch.Tensor],
                        name=None, learning_rate=None) -> List[torch.Tensor]:
        self._create_slots(var_list)
        lr = self._lr(learning_rate)
        out = []
        for var, g in zip(var_list, accum_grad_list):
            if g is None:
                g = torch.zeros_like(var)
            n = torch.linalg.vector_norm(g.float())
            g = g * (self._clip_norm / torch.maximum(n, torch.tensor(self._clip_norm, device=n.device)))
            self._apply_dense(g, var, lr)
            out.append(var)
        return out
