"""P1: node-owned sharding of event / span records across ranks."""

from __future__ import annotations

from typing import Tuple

import numpy as np

from ..collector.records import splitmix64_np


def owner_of_node(node_ids: np.ndarray, world: int) -> np.ndarray:
    """Rank owning each node: a hash, so node ids need not be dense or balanced."""
    if world <= 1:
        return np.zeros(np.shape(node_ids), dtype=np.int64)
    h = splitmix64_np(np.asarray(node_ids, dtype=np.uint64) ^ np.uint64(0x6E6F6465))  # "node"
    return (h % np.uint64(world)).astype(np.int64)


def shard(events: np.ndarray, spans: np.ndarray, rank: int, world: int) -> Tuple[np.ndarray, np.ndarray]:
    """This rank's events and spans (both keyed by node_id); order preserved."""
    if world <= 1:
        return events, spans
    ev = events[owner_of_node(events["node_id"], world) == rank]
    sp = spans[owner_of_node(spans["node_id"], world) == rank]
    return ev, sp


def trace_tagged(events: np.ndarray, supported_types=None) -> np.ndarray:
    """Mask of events that can match a span on another node (tier 1 = trace id only:
    pod ids are cluster-unique and svc+node is node-local, so tiers 2-4 never cross)."""
    m = (events["trace_h"] != 0) & (events["ts_ns"] != 0)
    if supported_types is not None:
        m &= np.isin(events["signal_type"], np.asarray(supported_types))
    return m
