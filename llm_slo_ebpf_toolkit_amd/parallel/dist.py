"""Process-group bring-up (one process per GPU; torchrun / torch.distributed.run env)."""

from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional


@dataclass
class DistEnv:
    rank: int = 0
    world: int = 1
    local_rank: int = 0

    @property
    def is_distributed(self) -> bool:
        return self.world > 1


def env() -> DistEnv:
    return DistEnv(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
                   int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: Optional[str] = None, device: Optional[int] = None, timeout_s: float = 600.0):
    """Initialise the default process group when WORLD_SIZE > 1; returns it (or None).

    ``backend`` defaults to ``nccl`` (RCCL on ROCm, over xGMI inside a node) when a GPU is
    visible and ``gloo`` otherwise. MASTER_ADDR defaults to 127.0.0.1 (the container
    hostname may not resolve)."""
    import datetime

    import torch
    import torch.distributed as dist

    e = env()
    if not e.is_distributed:
        return None
    if dist.is_initialized():
        return dist.group.WORLD
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    kw = {"timeout": datetime.timedelta(seconds=timeout_s)}
    if backend == "nccl":
        dev = e.local_rank if device is None else device
        torch.cuda.set_device(dev)
        kw["device_id"] = torch.device("cuda", dev)
    dist.init_process_group(backend, rank=e.rank, world_size=e.world, **kw)
    return dist.group.WORLD


def destroy() -> None:
    import torch.distributed as dist

    if dist.is_initialized():
        dist.destroy_process_group()
