"""CPU window engine: the numpy oracle of one window (pipeline/oracle.py) packaged with the
exact packet layout the GPU engine all-reduces (ops/csrc/bindings.cpp k_pack).

Two uses:

* the reference side of the multi-process tests -- ``gloo`` ranks run this engine on
  their shard, all-reduce the packets, and must reproduce the single-process window
  (parallel/ correctness by construction, no GPU needed);
* an explicit, loudly-selected CPU engine (``--device cpu``) for hosts without an MI355X
  (REF's deployment class, "config 1"). It is never a silent fallback: GPU hosts fail if
  the HIP extension is missing (ops.require_gpu_extension).
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np

from ..models.bayes import N_DOMAINS, LinearPosteriorModel, SufficientStats
from . import oracle
from .window import PACKET_LAYOUT

PACKET_LEN = sum(PACKET_LAYOUT)


@dataclass
class CpuWindowResult:
    packet: np.ndarray
    feat: np.ndarray
    post: np.ndarray
    pred: np.ndarray
    join: oracle.JoinResult


def build_packet(hist, status, misc, dbg, confusion, stats: SufficientStats) -> np.ndarray:
    p = np.zeros(PACKET_LEN, dtype=np.float64)
    o = 0
    parts = []
    st = np.zeros((32, 32))
    st[:16, :N_DOMAINS] = stats.elevated_sum
    st[16:, :N_DOMAINS] = stats.x_sum
    st[16:, 16:] = stats.xx
    cnt = np.zeros(16)
    cnt[:N_DOMAINS] = stats.count
    for arr in (hist, status, misc, dbg, confusion, st, cnt):
        parts.append(np.asarray(arr, dtype=np.float64).ravel())
    for part, n in zip(parts, PACKET_LAYOUT):
        assert part.size == n, (part.size, n)
        p[o:o + n] = part
        o += n
    return p


class CpuWindowEngine:
    def __init__(self, model: LinearPosteriorModel, window_ms: float = 2000.0, threshold: float = 0.7,
                 fanout: int = 3, group_mode: int = 1):
        self.model = model
        self.window_ms, self.threshold, self.fanout, self.group_mode = window_ms, threshold, fanout, group_mode

    def run(self, events: np.ndarray, spans: np.ndarray, n_groups: int, labels: Optional[np.ndarray] = None,
            n_local: Optional[int] = None, learn: bool = False, reduce_groups=None) -> CpuWindowResult:
        """One window. ``n_local``: events[n_local:] are imported (halo / remote trace-tagged)
        records: they join, but are not counted in the window's histograms/status/misc.

        ``reduce_groups(gsum, gcnt) -> (gsum, gcnt)``: global incident scope -- incident
        groups that span ranks are scored on the all-reduced per-group sums (the GPU
        pipeline's second, group-sum all-reduce); callers then pass ``labels`` only for the
        groups this rank owns so the confusion / statistics all-reduce counts each group once.
        """
        d = oracle.decode_events(events)
        n = events.shape[0]
        nl = n if n_local is None else int(n_local)
        loc = oracle.Decoded(*(getattr(d, f)[:nl] for f in ("ts", "val", "slot", "status", "pod", "pid",
                                                            "svcnode", "trace", "conn")))
        hist = oracle.histograms(loc)
        status = np.zeros((16, 3), dtype=np.int64)
        ok = loc.slot != oracle.NO_SLOT
        np.add.at(status, (loc.slot[ok].astype(np.int64), loc.status[ok].astype(np.int64)), 1)
        misc = np.zeros(PACKET_LAYOUT[2], dtype=np.int64)
        misc[0] = int((~ok).sum())
        misc[1] = int((loc.ts == 0).sum())
        misc[2:18] = oracle.value_sums_milli(loc)
        j = oracle.join(d, spans, n_groups, self.window_ms, self.threshold, self.fanout, self.group_mode)
        dbg = np.zeros(PACKET_LAYOUT[3], dtype=np.int64)
        dbg[0] = j.debug["candidates"]
        dbg[1] = j.debug["low_confidence"]  # overlap correction already applied (dbg[2] = 0)
        dbg[3] = j.debug["fanout_dropped"]
        dbg[4] = j.debug["spans_enriched"]
        gsum, gcnt = j.gsum, j.gcnt
        if reduce_groups is not None:
            gsum, gcnt = reduce_groups(gsum, gcnt)
        feat = oracle.group_features(gsum, gcnt).astype(np.float64)
        post = self.model.posteriors(feat)
        pred = np.argmax(self.model.logits(feat), axis=1) if n_groups else np.zeros(0, dtype=np.int64)
        conf = np.zeros((16, 16), dtype=np.int64)
        stats = SufficientStats()
        if labels is not None and n_groups:
            lab = np.asarray(labels[:n_groups], dtype=np.int64)
            m = lab >= 0
            np.add.at(conf, (lab[m], pred[m]), 1)
            if learn and m.any():
                stats.add(feat[m], lab[m])
        return CpuWindowResult(build_packet(hist, status, misc, dbg, conf, stats), feat.astype(np.float32), post,
                               pred, j)

    @staticmethod
    def unpack(packet: np.ndarray) -> Dict[str, np.ndarray]:
        from .window import unpack_packet

        return unpack_packet(packet)
