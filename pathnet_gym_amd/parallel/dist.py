"""Process-group bootstrap: one process per GPU, torch.distributed over RCCL.

Replaces the reference's TF gRPC parameter-server cluster
(``doom_pathnet.py:60-91``: ClusterSpec/Server/replica_device_setter).  There
is no PS: every rank holds a full replica of the 4-17 MB super-network in
HBM; ranks exchange only the fused per-update buffer (``comm.py``).

Launch: ``python -m torch.distributed.run --nproc-per-node N --master-addr
127.0.0.1 ...`` (env:// rendezvous).  Backend ``nccl`` is RCCL on ROCm;
``gloo`` is used for CPU runs/tests.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")
    # a real process group even at world size 1 (init_distributed(force=True)): every collective and the
    # multi-rank code paths (packed / overlapped all-reduce, RCCL barrier) run on a one-rank group -- how the
    # RCCL branches are exercised on a one-GPU box (tests/test_rccl_world1.py)
    forced: bool = False

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def enabled(self) -> bool:
        return self.world > 1 or self.forced

    # -- collectives (no-ops at world 1) -----------------------------------
    def all_reduce_(self, t: torch.Tensor):
        if self.enabled:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        if not self.enabled:
            return t.clone()
        flat = t.contiguous().reshape(-1)
        out = torch.empty(self.world * flat.numel(), dtype=t.dtype, device=t.device)
        if self.backend == "gloo":
            parts = list(out.chunk(self.world))
            dist.all_gather(parts, flat)
            out = torch.cat(parts)
        else:
            dist.all_gather_into_tensor(out, flat)
        return out.reshape((self.world * t.shape[0],) + tuple(t.shape[1:]))

    def broadcast_(self, t: torch.Tensor, src: int = 0):
        if self.enabled:
            dist.broadcast(t, src)
        return t

    def barrier(self):
        if self.enabled:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.local_rank])
            else:
                dist.barrier()

    def max_scalar(self, x: float) -> float:
        if not self.enabled:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def destroy(self):
        if self.enabled and dist.is_initialized():
            dist.destroy_process_group()


def init_distributed(device: Optional[str] = None, backend: Optional[str] = None, force: bool = False) -> DistContext:
    """Initialise from torchrun env vars (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*).  ``force`` (or PATHNET_DIST_FORCE=1):
    create the process group even at world size 1."""
    force = force or os.environ.get("PATHNET_DIST_FORCE") == "1"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    use_cuda = torch.cuda.is_available() if device is None else str(device).startswith("cuda")
    if use_cuda:
        ndev = torch.cuda.device_count()
        dev_idx = local_rank % max(1, ndev)          # ranks > devices only in the shared-GPU rehearsal
        torch.cuda.set_device(dev_idx)
        dev = torch.device("cuda", dev_idx)
    else:
        dev = torch.device("cpu")
    if world <= 1 and not force:
        return DistContext(0, 1, 0, "none", dev)
    # PATHNET_DIST_BACKEND=gloo lets several ranks share one GPU (test rehearsal); default RCCL ("nccl")
    be = backend or os.environ.get("PATHNET_DIST_BACKEND") or ("nccl" if use_cuda else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if world <= 1 and "MASTER_PORT" not in os.environ:
        # a forced one-rank group: bind port 0 for a free port, so concurrent forced jobs on one box do not collide
        import socket
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
            s.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(s.getsockname()[1])
    if not dist.is_initialized():
        if be == "nccl":
            dist.init_process_group(be, rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group(be, rank=rank, world_size=world)
    return DistContext(rank, world, dev.index if dev.type == "cuda" else local_rank, be, dev, forced=world <= 1)
