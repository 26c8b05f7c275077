"""Cross-shard record exchange for exact distributed joins (trace all-gather, P2 halo)."""

from __future__ import annotations

from typing import List, Optional, Tuple

import numpy as np

from ..signals import catalog
from .shard import trace_tagged


def allgather_records(local: np.ndarray, group=None, device=None) -> List[np.ndarray]:
    """All-gather variable-length structured record arrays (one collective for the sizes,
    one for the padded payload). Works on nccl (device tensors) and gloo (CPU tensors)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    dt = local.dtype
    dev = device if device is not None else torch.device("cpu")
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    cap = max(sizes) if sizes else 0
    if cap == 0:
        return [np.zeros(0, dtype=dt) for _ in range(world)]
    buf = np.zeros(cap, dtype=dt)
    buf[: local.shape[0]] = local
    t = torch.from_numpy(buf.view(np.uint8).copy()).to(dev)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t, group=group)
    return [o.cpu().numpy().view(dt)[:s].copy() for o, s in zip(outs, sizes)]


def with_remote_trace_events(local: np.ndarray, group=None, device=None) -> Tuple[np.ndarray, int]:
    """[local events..., trace-tagged events of every other rank...], n_local."""
    import torch.distributed as dist

    sup = [s.kernel_type for s in catalog.SIGNALS]
    mine = local[trace_tagged(local, sup)]
    parts = allgather_records(mine, group, device)
    me = dist.get_rank(group)
    remote = [p for r, p in enumerate(parts) if r != me and p.shape[0]]
    if not remote:
        return local, local.shape[0]
    return np.concatenate([local] + remote), local.shape[0]


class Halo:
    """P2 time halo for streaming windows: events of earlier windows whose timestamps lie
    within ``outer_ns`` of the current window's first span stay joinable. Imported halo
    events follow the window's own events (counted once, in their own window)."""

    def __init__(self, outer_ns: int, max_events: Optional[int] = None):
        self.outer_ns = int(outer_ns)
        self.max_events = max_events
        self._tail: Optional[np.ndarray] = None

    def extend(self, events: np.ndarray, spans: np.ndarray) -> Tuple[np.ndarray, int]:
        n_local = events.shape[0]
        merged = events
        if self._tail is not None and self._tail.shape[0] and spans.shape[0]:
            t0 = int(spans["ts_ns"][spans["ts_ns"] != 0].min()) if (spans["ts_ns"] != 0).any() else 0
            keep = self._tail[self._tail["ts_ns"] >= t0 - self.outer_ns]
            if keep.shape[0]:
                merged = np.concatenate([events, keep])
        # remember this window's tail (plus still-relevant older tail) for the next window
        if events.shape[0]:
            t_end = int(events["ts_ns"].max())
            pool = events if self._tail is None else np.concatenate([self._tail, events])
            tail = pool[pool["ts_ns"] >= t_end - self.outer_ns]
            if self.max_events is not None and tail.shape[0] > self.max_events:
                tail = tail[np.argsort(tail["ts_ns"], kind="stable")[-self.max_events:]]
            self._tail = tail
        return merged, n_local
