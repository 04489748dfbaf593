"""The reference's ``pathnet.py`` helper library on PyTorch tensors.

Every symbol of ``pathnet.py:10-196`` with the same
argument order.  TF variables become tensors; TF session/placeholder/assign
plumbing becomes in-place copies.  The GA operators draw from numpy's global
RNG by default, as in the reference, or from an explicit ``rng``.

The supervised module builders (``module``, ``module2``, ``conv_module``,
``nn_layer``) are the functional forms of the module kinds the batched
engines implement (``models/pathnet.py:trunk_forward_ref`` and the HIP
kernels); ``variable_summaries`` returns the TensorBoard statistics and
optionally forwards them to a ``MetricsLogger``.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from ..algo import ga as _ga


# -- parameter snapshot / restore (pathnet.py:10-18) -------------------------
def parameters_backup(var_list_to_learn: Sequence[torch.Tensor]) -> List[torch.Tensor]:
    """Detached copies of every tensor (pathnet.py:10-14)."""
    return [v.detach().clone() for v in var_list_to_learn]


def parameters_update(sess, var_list, var_update_ops_unused, var_list_backup) -> None:
    """Restore tensors from a backup in place (pathnet.py:16-18).

    ``sess`` and the assign-op list are accepted for call-site compatibility;
    ``var_list`` are the tensors to overwrite.
    """
    with torch.no_grad():
        for v, b in zip(var_list, var_list_backup):
            v.copy_(torch.as_tensor(b, dtype=v.dtype, device=v.device))


# -- genotype storage (pathnet.py:20-30) -------------------------------------
def geopath_initializer(L: int, M: int, device="cpu") -> torch.Tensor:
    """L x M mask, all modules active (pathnet.py:25-30 creates tf.Variable(1.0) each)."""
    return torch.ones(L, M, device=device)


def geopath_insert(sess, geopath, geopath_update_ops_unused, candi, L: int, M: int) -> None:
    """Write genotype ``candi`` [L,M] into ``geopath`` in place (pathnet.py:20-23).

    ``geopath`` is a [L,M] tensor/ndarray or an object with ``set_geopath``
    (the compat networks) -- one copy instead of L*M session runs.
    """
    c = np.asarray(candi, dtype=np.float32)[:L, :M]
    if hasattr(geopath, "set_geopath"):
        geopath.set_geopath(c)
    elif isinstance(geopath, torch.Tensor):
        with torch.no_grad():
            geopath[:L, :M].copy_(torch.from_numpy(c))
    else:
        geopath[:L, :M] = c


# -- GA operators (pathnet.py:32-87) -----------------------------------------
def mutationDown(geopath, L, M, N, rng=np.random):   # noqa: N802  (reference name)
    return _ga.mutation_down(geopath, L, M, N, rng)


def mutation(geopath, L, M, N, rng=np.random):
    return _ga.mutation(geopath, L, M, N, rng)


def select_two_candi(M, rng=np.random):
    return _ga.select_two_candi(M, rng)


def get_geopath(L, M, N, rng=np.random):
    return _ga.get_geopath(L, M, N, rng)


# -- variable factories (pathnet.py:90-108) ----------------------------------
def weight_variable(shape, device="cpu", generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """truncated_normal(stddev=0.1): resample outside +-2 sigma (pathnet.py:90-93)."""
    t = torch.empty(tuple(shape))
    torch.nn.init.trunc_normal_(t, mean=0.0, std=0.1, a=-0.2, b=0.2, generator=generator)
    return t.to(device).requires_grad_(True)


def bias_variable(shape, device="cpu") -> torch.Tensor:
    """constant 0.1 (pathnet.py:95-98)."""
    return torch.full(tuple(shape), 0.1, device=device).requires_grad_(True)


def module_weight_variable(shape, device="cpu") -> List[torch.Tensor]:
    return [weight_variable(shape, device)]


def module_bias_variable(shape, device="cpu") -> List[torch.Tensor]:
    return [bias_variable(shape, device)]


def variable_summaries(var: torch.Tensor, name: str = "", logger=None, step: int = 0) -> dict:
    """mean / stddev / max / min / histogram of a tensor (pathnet.py:110-120)."""
    v = var.detach().float().reshape(-1)
    hist, edges = np.histogram(v.cpu().numpy(), bins=30)
    out = {"mean": float(v.mean()), "stddev": float(v.std(unbiased=False)), "max": float(v.max()),
           "min": float(v.min()), "histogram": hist.tolist(), "edges": edges.tolist()}
    if logger is not None:
        logger.log("summary", name=name, step=step, **{k: out[k] for k in ("mean", "stddev", "max", "min")})
    return out


# -- module kinds (pathnet.py:122-196) ---------------------------------------
def module(input_tensor, weights, biases, layer_name: str = "", act: Callable = F.relu):
    """FC module act(x W + b) (pathnet.py:122-135)."""
    w = weights[0] if isinstance(weights, (list, tuple)) else weights
    b = biases[0] if isinstance(biases, (list, tuple)) else biases
    return act(input_tensor @ w + b)


def module2(i: int, input_tensor, weights, biases, layer_name: str = "", act: Callable = F.relu):
    """Heterogeneous module by index (pathnet.py:137-168): i%3 == 0 skip, 1 fc+act, 2 residual."""
    kind = i % 3
    if kind == 0:
        return input_tensor
    y = module(input_tensor, weights, biases, layer_name, act)
    return y if kind == 1 else y + input_tensor


def conv_module(input_tensor, weights, biases, stride: int, layer_name: str = "", act: Callable = F.relu):
    """NHWC VALID conv + bias + act, TF weight layout [kh,kw,cin,cout] (pathnet.py:170-183)."""
    w = weights[0] if isinstance(weights, (list, tuple)) else weights
    b = biases[0] if isinstance(biases, (list, tuple)) else biases
    y = F.conv2d(input_tensor.permute(0, 3, 1, 2), w.permute(3, 2, 0, 1), b, stride=stride)
    return act(y.permute(0, 2, 3, 1))


def nn_layer(input_tensor, weights, biases, layer_name: str = ""):
    """Linear output layer, no activation (pathnet.py:185-196)."""
    w = weights[0] if isinstance(weights, (list, tuple)) else weights
    b = biases[0] if isinstance(biases, (list, tuple)) else biases
    return input_tensor @ w + b
