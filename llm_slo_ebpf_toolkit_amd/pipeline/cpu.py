"""CPU window engines: the numpy oracle of one window (pipeline/oracle.py) packaged with the
exact packet layout the GPU engine all-reduces (ops/csrc/engine.hip k_pack).

* ``CpuWindowEngine`` -- one window of 64-byte EVENT/SPAN records: the reference side of the
  record-level tests;
* ``CpuRingEngine`` -- the native ``WindowEngine``'s contract (ring byte ranges in, packet and
  per-incident results out, halo, group sharding, the collectives over a gloo group). It is the
  engine of ``agent --engine cpu`` (hosts without an MI355X, REF's deployment class, "config 1")
  and of the multi-process agent tests, where ``gloo`` ranks must reproduce the single-process
  window. It is never a silent fallback: GPU hosts fail if the HIP extension is missing
  (ops.require_gpu_extension).
"""

from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np

from ..collector import records
from ..models.bayes import N_DOMAINS, LinearPosteriorModel, SufficientStats, app_counts, soft_labels
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


STATS_OFF, STATS_LEN = sum(PACKET_LAYOUT[:5]), PACKET_LAYOUT[5] + PACKET_LAYOUT[6]  # sufficient statistics


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
        pred = self.model.predict(feat) if n_groups else np.zeros(0, dtype=np.int64)
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


# ---------------------------------------------------------------------------------------
# the native engine's window contract on the CPU (agent --engine cpu, multi-process tests)
# ---------------------------------------------------------------------------------------

def _read(addr: int, n: int) -> np.ndarray:
    import ctypes

    if n <= 0:
        return np.zeros(0, dtype=np.uint8)
    return np.ctypeslib.as_array((ctypes.c_uint8 * int(n)).from_address(int(addr))).copy()


def _gather(segs) -> np.ndarray:
    parts = [_read(a, n) for a, n in segs]
    return np.concatenate(parts) if parts else np.zeros(0, dtype=np.uint8)


def shard_owner(svcnode: np.ndarray, world: int) -> np.ndarray:
    """decode.hip shard_owns: service s >= 1 -> GPU (s - 1) % world, no service -> GPU 0."""
    svc = (np.asarray(svcnode, dtype=np.uint32) >> np.uint32(16)).astype(np.int64)
    return np.where(svc > 0, (svc - 1) % max(1, world), 0)


class CpuRingEngine:
    """The native ``WindowEngine``'s window contract (ops/csrc/engine.h) evaluated by the numpy
    oracle on the host: the same ring byte ranges in (framed BPF ring records, user-space
    records, spans), the same packet, per-incident results, busy-record stop, halo, group
    sharding and -- with a ``torch.distributed`` group (gloo) -- the same collectives: the
    packet all-reduce (ring accounting excluded), the all-gather of every rank's incident
    results and of the trace-tagged exchange blocks.

    Selected explicitly (``agent --engine cpu``; the multi-process tests), never as a silent
    fallback. The oracle join is O(spans x rows): a reference engine for small windows, not a
    production path at node event rates."""

    def __init__(self, device: int = 0, sig_cap: int = 1 << 20, span_cap: int = 16384, group_cap: int = 64, user_cap: int = 1 << 18,
                 n_buffers: int = 3, window_ms: float = 2000.0, threshold: float = 0.7, fanout: int = 3,
                 group_mode: int = 1, n_dom: int = N_DOMAINS, ttft_slo_ms: float = 800.0, halo_ms: float = 0.0,
                 import_cap: int = 0, xchg_cap: int = 0, shard_rank: int = 0, shard_world: int = 1, group=None,
                 halo_windows: int = 3, split_rings: bool = False, **_native_only):
        from ..parallel.exchange import ExchangeModel, torch_allgather

        self.sig_cap, self.span_cap, self.group_cap, self.user_cap = sig_cap, span_cap, group_cap, user_cap
        self.buffers = int(n_buffers)
        self.window_ms_, self.threshold, self.fanout, self.group_mode = window_ms, threshold, fanout, group_mode
        self.n_dom, self.ttft_slo_ms = n_dom, float(ttft_slo_ms)
        self.shard_rank, self.shard_world = int(shard_rank), int(shard_world)
        self.split_rings = bool(split_rings)
        self.group = group
        if group is not None:
            import torch.distributed as dist

            self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        else:
            self.rank, self.world = 0, 1
        self.xm = ExchangeModel(self.rank, self.world, halo_ms, import_cap, xchg_cap if self.world > 1 else 0,
                                torch_allgather(group) if group is not None else None, halo_windows=halo_windows)
        self.table, self.tmap = oracle.CtxTable(), oracle.TraceMap()
        self.pod_sn: Dict[int, int] = {}
        self.model = None
        self.app = None  # application evidence (set_app_model)
        self.win: Dict[int, dict] = {}
        self._totals = np.zeros(PACKET_LEN)
        self._stats_acc = np.zeros(STATS_LEN)
        self.windows_folded = 0
        self.graphs = 0
        self.staged_bytes = self.direct_bytes = 0
        self.host_issue_us = self.host_wait_us = self.host_dma_issue_us = self.host_launch_us = 0.0
        self.host_pre_us = self.host_tail_us = 0.0
        self.host_dma_split_us = [0.0, 0.0, 0.0, 0.0]

    @property
    def has_comm(self) -> bool:
        return self.group is not None and self.world > 1

    # ---- setup ------------------------------------------------------------------------------
    def register_host(self, addr: int, n: int) -> bool:
        return True

    def set_model_bytes(self, b) -> None:
        from ..ops.engine import model_from_bytes

        self.model_image = np.ascontiguousarray(b, dtype=np.uint8).copy()
        self.model = model_from_bytes(self.model_image)

    def model_bytes(self) -> np.ndarray:
        return self.model_image.copy()

    def set_app_model(self, b) -> None:
        from ..ops.engine import app_from_bytes

        self.app = app_from_bytes(b, self.n_dom)

    def set_p0(self, p0) -> None:
        pass

    def set_pods(self, pods, sn) -> None:
        self.pod_sn.update(zip(np.asarray(pods).tolist(), np.asarray(sn).tolist()))

    def init_comm(self, *a) -> None:
        raise RuntimeError("the CPU engine communicates over its torch.distributed group (gloo)")

    # ---- per window -------------------------------------------------------------------------
    def submit(self, k: int, kernel, user, spans, n_groups: int, labels, bases, with_labels: bool, learn: bool,
               user_rec: int) -> None:
        t0 = time.perf_counter()
        framed = _gather(kernel)
        words = records.REC_STRIDE // 4
        fr = framed.view(np.uint32).reshape(-1, words) if len(framed) else np.zeros((0, words), np.uint32)
        busy = np.nonzero(fr[:, 0] & np.uint32(records.RB_BUSY))[0] if len(fr) else np.zeros(0, np.int64)
        # in rows, like the device: the busy batch's first slot
        first_busy = int(busy[0]) * records.BATCH_SLOTS if len(busy) else -1
        oracle.apply_ring_defs(framed, self.table, self.tmap, self.pod_sn)
        if first_busy >= 0:  # the engine stops at the first record still being written
            fr = fr.copy()
            fr[int(busy[0]):, 0] = np.uint32(records.RB_BUSY | records.REC_PAYLOAD)
            framed = fr.view(np.uint8).reshape(-1)
        ub = _gather(user)
        udt = {64: records.EVENT, 32: records.USER32, 24: records.USER24, 16: records.USER16}[int(user_rec)]
        u = ub.view(udt) if len(ub) else np.zeros(0, dtype=udt)
        d = oracle.decode_window(framed, u, self.table, self.tmap, bases, pod_sn=self.pod_sn)
        hdr, sl = records.framed_slots(framed) if len(fr) else (np.zeros(0, np.uint32), np.zeros((0, 4), np.uint32))
        valid_k = (hdr == records.REC_PAYLOAD) & ((sl[:, 1] & np.uint32(0xFF)) < records.DEF_FIRST)
        other = 0
        # USER16 continuation slots (a traced record's trace) are rows but not records
        u_rec = u["pid_sig"] != np.uint32(records.USER16_CONT) if u.dtype == records.USER16 else np.ones(len(u), bool)
        is_rec = np.concatenate([valid_k, u_rec])
        if self.shard_world > 1 and not self.split_rings:  # split rings: routed by the producers
            mine = shard_owner(d.svcnode, self.shard_world) == self.shard_rank
            drop = is_rec & ~mine
            other = int(drop.sum())
            d = _holes(d, drop)
            is_rec = is_rec & ~drop
        events = int(valid_k.sum()) + int(u_rec.sum()) - other
        sp = _gather(spans)
        spr = oracle.spans_native(sp.view(records.SPAN) if len(sp) else np.zeros(0, records.SPAN))
        counted = (spr["flags"] & np.uint32(records.SPAN_NO_SLI)) == 0  # first-token records count once
        G = int(n_groups)
        grp_local = spr["group_id"].astype(np.int64)
        if self.shard_world > 1:
            mine_sp = grp_local % self.shard_world == self.shard_rank
            spr["ts_ns"] = np.where(mine_sp, spr["ts_ns"], 0)
            grp_local = grp_local // self.shard_world
            spr["group_id"] = grp_local.astype(spr["group_id"].dtype)
        else:
            mine_sp = np.ones(len(spr), bool)
        n_loc = len(d.ts)
        res = self.xm.window(d, spr, G, window_ms=self.window_ms_, threshold=self.threshold, fanout=self.fanout,
                             group_mode=self.group_mode)
        hist = oracle.histograms(d)
        status = np.zeros((16, 3), dtype=np.int64)
        ok = d.slot != oracle.NO_SLOT
        np.add.at(status, (d.slot[ok].astype(np.int64), d.status[ok].astype(np.int64)), 1)
        misc = np.zeros(PACKET_LAYOUT[2], dtype=np.int64)
        misc[0] = int(((~ok) & is_rec).sum())
        misc[1] = int(((d.ts == 0) & is_rec).sum())
        misc[2:18] = oracle.value_sums_milli(d)
        dbg = np.zeros(PACKET_LAYOUT[3], dtype=np.int64)
        dbg[0] = res.debug["candidates"]
        dbg[1] = res.debug["low_confidence"]
        dbg[3] = res.debug["fanout_dropped"]
        dbg[4] = res.debug["spans_enriched"]
        dbg[5], dbg[6] = self.xm.xchg_dropped, self.xm.import_dropped
        feat = res.feat.astype(np.float32)
        f64 = feat.astype(np.float64)
        D = self.n_dom
        post = np.zeros((G, 16))
        pred = np.zeros(G, np.int32)
        gconf = np.zeros(G)
        evbits = np.zeros((G, 16), np.uint32)
        okg = mine_sp & (grp_local >= 0) & (grp_local < G)
        app = app_counts(spr, G, mine=okg, groups=grp_local)
        if G and self.model is not None:
            self.model.app = self.app
            st = self.app.state(app, feat) if self.app is not None else None
            post[:, :D] = self.model.posteriors(f64, st)
            pred = self.model.predict(f64, st).astype(np.int32)
            gconf = post[np.arange(G), pred]
            evbits[:, :D] = self.model.evidence_bits(f64, st)
        conf = np.zeros((16, 16), dtype=np.int64)
        stats = SufficientStats()
        if labels is not None and G:
            lab = np.asarray(labels, dtype=np.int64)[:G]
            m = lab >= 0
            if with_labels:
                np.add.at(conf, (lab[m] & 0xFF, pred[m]), 1)
            if learn and m.any():
                stats.add(f64[m], soft_labels(lab[m]))
        sli = np.zeros((G, 2), np.uint32)
        late = np.zeros((G, 2), np.uint32)
        breach = spr["ttft_ms"] > np.float32(self.ttft_slo_ms)
        is_late = breach & ((spr["flags"] & np.uint32(records.SPAN_LATE)) != 0)
        ok = okg & counted
        np.add.at(sli[:, 0], grp_local[ok & ~is_late], 1)
        np.add.at(sli[:, 1], grp_local[ok & breach & ~is_late], 1)
        np.add.at(late[:, 0], grp_local[ok & is_late], 1)
        ring = np.zeros(PACKET_LAYOUT[7])
        ring[:7] = (first_busy, 0, 0, 0, 0, events, other)
        pk = build_packet(hist, status, misc, dbg, conf, stats)
        pk[PACKET_LEN - PACKET_LAYOUT[7]:] = ring
        out = {"post": post, "conf": gconf, "feat": feat, "pred": pred, "evbits": evbits, "sli": sli, "app": app,
               "late": late}
        outs = [out]
        if self.has_comm:
            import torch
            import torch.distributed as dist

            t = torch.from_numpy(pk[:PACKET_LEN - PACKET_LAYOUT[7]].copy())
            dist.all_reduce(t, group=self.group)
            pk[:PACKET_LEN - PACKET_LAYOUT[7]] = t.numpy()
            outs = [None] * self.world
            dist.all_gather_object(outs, out, group=self.group)
        self._totals += pk
        if learn:  # the node-wide statistics of learning windows (the device folds them in k_refit_nb)
            self._stats_acc += pk[STATS_OFF:STATS_OFF + STATS_LEN]
        ms = 1e3 * (time.perf_counter() - t0)
        self.win[k % max(1, self.buffers)] = {"k": k, "packet": pk, "res": out, "all": outs, "ms": ms,
                                             "rows": (n_loc, res.n_rows)}

    def _w(self, k: int) -> dict:
        w = self.win.get(k % max(1, self.buffers))
        if w is None or w["k"] != k:
            raise KeyError(f"window {k} is not held (only the last {self.buffers})")
        return w

    def h2d_done(self, k: int) -> bool:
        return True

    def wait_h2d(self, k: int) -> None:
        pass

    def query(self, k: int) -> bool:
        return True

    def wait(self, k: int) -> None:
        self._w(k)

    def packet(self, k: int) -> np.ndarray:
        return self._w(k)["packet"].copy()

    @staticmethod
    def _cut(r: dict, G: int) -> dict:
        return {key: np.asarray(v)[:G].copy() for key, v in r.items()}

    def results(self, k: int, n_groups: int) -> dict:
        return self._cut(self._w(k)["res"], n_groups)

    def results_all(self, k: int, n_groups: int) -> list:
        return [self._cut(r, n_groups) for r in self._w(k)["all"]]

    def window_ms(self, k: int):
        ms = self._w(k)["ms"]
        return ms, ms

    def copy_ms(self, k: int):
        return [0.0, 0.0]

    def inject_remote(self, blocks, stride, world, me) -> None:
        from ..parallel.exchange import parse_block

        b = np.ascontiguousarray(blocks, dtype=np.uint8)
        for r in range(world):
            if r != me:
                self.xm.injected = oracle.concat(self.xm.injected, parse_block(b[r * stride:(r + 1) * stride]))

    def import_state(self):
        return []

    # ---- totals / state -----------------------------------------------------------------------
    def totals(self) -> np.ndarray:
        return self._totals.copy()

    def reset_totals(self) -> None:
        self._totals[:] = 0

    def stats_acc(self) -> np.ndarray:
        return self._stats_acc.copy()

    def restore(self, stats, model, folded) -> None:
        if stats is not None and len(stats) == STATS_LEN:
            self._stats_acc = np.asarray(stats, dtype=np.float64).copy()
        if len(model):
            self.set_model_bytes(model)

    # The host engine scores with the model image it was given: the device refit (k_refit_nb,
    # rebuilding the tables from the all-reduced statistics) has no counterpart here, and the image
    # a trainer restores is already the host-fitted model (models/train.py), which the device refit
    # reproduces (__graft_entry__.smoke checks that equality on the GPU).
    def set_refit(self, alpha: float, prior_pseudo: float, inv_temp: float, min_count: float, cap_dom: int = -1,
                  ceil: float = 1.0) -> None:
        self.refit_params = (float(alpha), float(prior_pseudo), float(inv_temp), float(min_count), int(cap_dom),
                             float(ceil))

    def refit_now(self) -> None:
        pass

    def set_device_refit(self, on: bool) -> None:
        pass

    def sync(self) -> None:
        pass

    def close(self) -> None:
        self.win.clear()


def _holes(d: oracle.Decoded, m: np.ndarray) -> oracle.Decoded:
    """Rows ``m`` become holes: no timestamp, no signal, no identity (decode.hip hole rows)."""
    out = oracle.Decoded(*(getattr(d, f).copy() for f in oracle.Decoded.__dataclass_fields__))
    for f, z in (("ts", 0), ("val", 0), ("slot", oracle.NO_SLOT), ("status", 0), ("pod", 0), ("pid", 0),
                 ("svcnode", 0), ("trace", 0), ("conn", 0)):
        getattr(out, f)[m] = z
    return out
