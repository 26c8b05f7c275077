"""K6 batched retry-storm counts (ops/csrc/storm.hip) + numpy oracle.

``windowed_counts(pod_keys, ts_ns)`` returns, per event in input order, the value
REF ``RetryStormDetector.Record`` would leave for that pod if the events arrived in
(pod, ts) order (pkg/correlation/retry_storm.go:46-60): the number of the pod's events in
[ts - window, ts] up to and including this one. Sorting runs on the device (two stable
``torch.sort`` passes), the counting in the HIP kernel.
"""

from __future__ import annotations

from typing import Tuple

import numpy as np

from ..correlation.retry_storm import DEFAULT_STORM_THRESHOLD, DEFAULT_STORM_WINDOW_NS


def windowed_counts_np(pod_keys: np.ndarray, ts_ns: np.ndarray, window_ns: int = DEFAULT_STORM_WINDOW_NS,
                       threshold: int = DEFAULT_STORM_THRESHOLD) -> Tuple[np.ndarray, int]:
    keys = np.asarray(pod_keys, dtype=np.int64)
    ts = np.asarray(ts_ns, dtype=np.int64)
    order = np.lexsort((ts, keys))
    k, t = keys[order], ts[order]
    n = len(k)
    seg = np.searchsorted(k, k, side="left")
    lo = np.empty(n, dtype=np.int64)
    for i in range(n):  # oracle clarity over speed
        lo[i] = seg[i] + np.searchsorted(t[seg[i]:i + 1], t[i] - window_ns, side="left")
    c_sorted = np.arange(n) - lo + 1
    counts = np.empty(n, dtype=np.int64)
    counts[order] = c_sorted
    return counts, int((c_sorted >= threshold).sum())


def windowed_counts(pod_keys, ts_ns, window_ns: int = DEFAULT_STORM_WINDOW_NS,
                    threshold: int = DEFAULT_STORM_THRESHOLD, device: int = 0):
    """Device path. Accepts numpy arrays or int64 tensors; returns (counts[int64], n_storm_events)."""
    import torch

    from . import load

    mod = load(device)
    dev = torch.device("cuda", device)
    keys = torch.as_tensor(np.asarray(pod_keys, dtype=np.int64) if not torch.is_tensor(pod_keys) else pod_keys,
                           device=dev)
    ts = torch.as_tensor(np.asarray(ts_ns, dtype=np.int64) if not torch.is_tensor(ts_ns) else ts_ns, device=dev)
    with torch.cuda.device(dev):
        o1 = torch.sort(ts, stable=True).indices
        o2 = torch.sort(keys[o1], stable=True).indices
        order = o1[o2]
        counts_sorted, tally = mod.storm_counts(keys[order].contiguous(), ts[order].contiguous(), int(window_ns),
                                                int(threshold))
        counts = torch.empty_like(counts_sorted)
        counts[order] = counts_sorted
    return counts.long().cpu().numpy(), int(tally.item())
