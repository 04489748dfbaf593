"""Race / divergence detection for the replicated-state design.

Every rank holds a full replica of the super-network, the optimizer slots and
the GA state, and must stay bit-identical to the others: the weights because
all ranks apply the same all-reduced gradient, the GA because it is a
deterministic function of the all-reduced fitness vector.  Any race --
a kernel reading a buffer before a collective finished, a non-deterministic
reduction feeding the GA, a rank skipping a step -- shows up as replicas that
drift apart.  The reference had exactly this class of bug with no detector
(lost global_step updates, Hogwild RMSProp, genotype swaps mid-rollout;
SURVEY.md section 5).

``state_digest`` reduces the replicated state to a few numbers (exact
checksums of the weights and RMSProp slots computed on device, a hash of
genotypes / frozen mask / fitness / counters); ``check_replicas`` all-gathers
the digests (one tiny collective) and raises ``DivergenceError`` naming the
ranks that disagree with rank 0.  The trainer runs it every
``check_every`` updates (``--check_every``).
"""
from __future__ import annotations

import hashlib
from typing import Dict, List

import numpy as np
import torch


class DivergenceError(RuntimeError):
    pass


def _tensor_checksum(t: torch.Tensor) -> List[float]:
    """Order-sensitive exact checksum: int64 sum of the raw fp32 bit patterns, weighted and plain."""
    bits = t.detach().contiguous().view(torch.int32).to(torch.int64)
    idx = torch.arange(bits.numel(), device=bits.device, dtype=torch.int64) % 65521 + 1
    s1 = int(bits.sum())
    s2 = int((bits * idx).sum())
    return [float(s1 % (1 << 52)), float(s2 % (1 << 52))]


def state_digest(trainer) -> torch.Tensor:
    """[8] float64 digest of the state that must be identical on every rank."""
    flat = trainer.model.store.flat
    vals = _tensor_checksum(flat) + _tensor_checksum(trainer.opt.ms)
    pop = trainer.pop
    h = hashlib.sha256()
    for a in (pop.genotypes, pop.frozen, pop.fitness):
        h.update(np.ascontiguousarray(a).tobytes())
    h.update(np.array([pop.generation, trainer.global_step, trainer.updates, trainer.task_idx],
                      np.int64).tobytes())
    d = h.digest()
    vals += [float(int.from_bytes(d[i:i + 6], "little")) for i in (0, 6, 12, 18)]
    return torch.tensor(vals, dtype=torch.float64)


def check_replicas(trainer) -> Dict[str, object]:
    ctx = trainer.ctx
    dig = state_digest(trainer)
    if not ctx.enabled:
        return {"ok": True, "digest": dig.tolist()}
    dev = ctx.device
    allg = ctx.all_gather(dig.to(dev)[None]).cpu()       # [world, 8]
    bad = [r for r in range(ctx.world) if not torch.equal(allg[r], allg[0])]
    if bad:
        fields = ["weights", "weights_w", "rms", "rms_w", "ga0", "ga1", "ga2", "ga3"]
        diff = {r: [fields[i] for i in range(8) if allg[r, i] != allg[0, i]] for r in bad}
        raise DivergenceError(f"replicated state diverged from rank 0 on ranks {bad}: {diff} "
                              f"(update {trainer.updates})")
    return {"ok": True, "digest": dig.tolist()}
