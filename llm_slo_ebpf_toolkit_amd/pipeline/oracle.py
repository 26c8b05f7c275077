"""CPU reference ("oracle") of one GPU window, bit-faithful to the kernels' contracts.

Given the same 64-byte EVENT/SPAN records the GPU consumes, recompute with plain numpy
and REF's scalar semantics (correlation/match.py, correlation/correlator.py):
decode (float32 values exactly as the kernel rounds them), per-span tiers, top-3
candidate keys, merged attributes, confidence, debug counters, incident-group features,
histograms and posteriors. Tests compare the GPU outputs against this (exact for keys,
tiers, counts, predictions; tolerance for float sums whose order differs).
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np

from ..collector import records
from ..signals import catalog
from ..utils.timeutil import MS

NO_SLOT = 255
SIG_BITS = 27
TIER_CONF = (1.0, 0.9, 0.8, 0.65)


@dataclass
class Decoded:
    ts: np.ndarray
    val: np.ndarray
    slot: np.ndarray
    status: np.ndarray
    pod: np.ndarray
    pid: np.ndarray
    svcnode: np.ndarray
    trace: np.ndarray
    conn: np.ndarray


def decode_events(ev: np.ndarray) -> Decoded:
    type_slot = np.full(65536, NO_SLOT, dtype=np.uint8)
    scale32 = np.zeros(16, dtype=np.float32)
    for s in catalog.SIGNALS:
        type_slot[s.kernel_type] = s.slot
        scale32[s.slot] = np.float32(s.decode_scale)
    st = ev["signal_type"].astype(np.int64)
    slot = type_slot[st]
    ok = slot != NO_SLOT
    val = ev["value"].astype(np.float64).astype(np.float32)
    sc = scale32[np.where(ok, slot, 0)].astype(np.float64)
    val = np.where(ok, (ev["value"].astype(np.float64) * sc).astype(np.float32), val)
    warn = np.array([s.warn for s in catalog.SIGNALS], dtype=np.float32)
    err = np.array([s.error for s in catalog.SIGNALS], dtype=np.float32)
    sl = np.where(ok, slot, 0)
    status = np.where(val >= err[sl], 2, np.where(val >= warn[sl], 1, 0)).astype(np.uint8)
    status = np.where(ok, status, 0).astype(np.uint8)
    conn = ev["conn_h"].copy()
    derived = records.conn_hash_np(ev["src_port"], ev["dst_port"], ev["dst_ip"])
    conn = np.where(conn == 0, derived, conn)
    svcnode = (ev["svc_id"].astype(np.uint32) << np.uint32(16)) | ev["node_id"].astype(np.uint32)
    return Decoded(ev["ts_ns"].astype(np.int64), val, slot, status, ev["pod_id"].astype(np.uint32),
                   ev["pid"].astype(np.uint32), svcnode, ev["trace_h"].astype(np.uint64), conn.astype(np.uint64))


class CtxTable:
    """Sparse view of the device context table: (ids, rows) pairs, later pairs win (the patch
    order of the window engine); absent ids read the all-zero row."""

    def __init__(self, ids=None, rows=None):
        self.map = {}
        if ids is not None:
            self.add(ids, rows)

    def add(self, ids, rows) -> "CtxTable":
        for i, r in zip(np.asarray(ids).tolist(), np.asarray(rows, dtype=np.uint32).reshape(-1, 4).tolist()):
            self.map[int(i)] = tuple(r)
        return self

    def rows(self, cid: np.ndarray) -> np.ndarray:
        out = np.zeros((cid.shape[0], 4), dtype=np.uint32)
        for j, c in enumerate(cid.tolist()):
            r = self.map.get(int(c))
            if r is not None:
                out[j] = r
        return out


def decode_w16(ev: np.ndarray, table: CtxTable, bases) -> Decoded:
    """k_decode_wire on EVENT16 records: ts = bases[tag] + ts_off, context rows from the table."""
    type_slot = np.full(256, NO_SLOT, dtype=np.uint8)
    for s in catalog.SIGNALS:
        if s.kernel_type < 256:
            type_slot[s.kernel_type] = s.slot
    ct = ev["ctx_type"].astype(np.uint32)
    st = (ct & np.uint32(0xFF)).astype(np.int64)
    slot = type_slot[st]
    val = (ev["value_milli"].astype(np.float64) * 1e-3).astype(np.float32)
    warn = np.array([s.warn for s in catalog.SIGNALS], dtype=np.float32)
    err = np.array([s.error for s in catalog.SIGNALS], dtype=np.float32)
    ok = slot != NO_SLOT
    sl = np.where(ok, slot, 0)
    status = np.where(ok, np.where(val >= err[sl], 2, np.where(val >= warn[sl], 1, 0)), 0).astype(np.uint8)
    row = table.rows((ct >> np.uint32(8)).astype(np.int64))
    off = ev["ts_off"].astype(np.int64)
    b = np.array((list(bases) + [0, 0, 0, 0])[:4], dtype=np.int64)
    tag = (ev["trace_id"].astype(np.uint32) >> np.uint32(30)).astype(np.int64)
    ts = np.where(off == 0xFFFFFFFF, 0, b[tag] + off)
    trace = ev["trace_id"].astype(np.uint32) & np.uint32((1 << 30) - 1)
    return Decoded(ts, val, slot, status, row[:, 0], row[:, 1], row[:, 3], trace.astype(np.uint64),
                   row[:, 2].astype(np.uint64))


class TraceMap:
    """Host mirror of the engine's trace-id table (mislo_common.h TraceIds): the probes' TRACE
    definitions name the hash behind each kernel trace id; kernel records decode to the hash,
    user-space records and spans carry hashes already."""

    def __init__(self):
        self.m: Dict[int, int] = {}  # kernel trace id -> hash

    def hashes(self, ids: np.ndarray) -> np.ndarray:
        return np.array([self.m.get(int(i), 0) if i else 0 for i in np.asarray(ids).tolist()], dtype=np.uint64)


def apply_ring_defs(framed: np.ndarray, table: CtxTable, tmap: TraceMap, pod_sn: Dict[int, int]) -> None:
    """k_ring_defs: context rows (svc|node from pod metadata) and trace ids of a framed window."""
    hdr, sl = records.framed_slots(framed)
    p = sl[hdr == records.REC_PAYLOAD]
    t = p[:, 1] & 0xFF
    for c32, ct, pod, pid in p[t == records.DEF_CTX].tolist():
        table.map[ct >> 8] = (pod, pid, c32, pod_sn.get(pod, 0))
    for tid, _ct, lo, hi in p[t == records.DEF_TRACE].tolist():
        if 0 < tid < records.KERNEL_TRACE_LIMIT:
            tmap.m[tid] = lo | (hi << 32)


def decode_user32(u: np.ndarray, pod_sn: Dict[int, int]) -> Decoded:
    """k_decode_window on USER32 rows: fixed-point value, svc|node from the pod table, no connection."""
    type_slot = np.full(256, NO_SLOT, dtype=np.uint8)
    for s in catalog.SIGNALS:
        if s.kernel_type < 256:
            type_slot[s.kernel_type] = s.slot
    slot = type_slot[u["signal_type"].astype(np.int64)]
    val = (u["value_milli"].astype(np.float64) * 1e-3).astype(np.float32)
    sn = np.array([pod_sn.get(int(p), 0) for p in u["pod_id"].tolist()], dtype=np.uint32)
    n = len(u)
    return Decoded(u["ts_ns"].astype(np.int64), val, slot, status_of(val, slot), u["pod_id"].astype(np.uint32),
                   u["pid"].astype(np.uint32), sn, u["trace_h"].astype(np.uint64), np.zeros(n, np.uint64))


def decode_user24(u: np.ndarray, pod_sn: Dict[int, int], base: int) -> Decoded:
    """k_decode_window on USER24 rows: USER32's decode with the packed pid / type / pod id and the
    timestamp nearest ``base`` (the window's newest epoch base)."""
    return decode_user32(records.user24_to_user32(u, base), pod_sn)


def decode_user16(u: np.ndarray, pod_sn: Dict[int, int], base: int) -> Decoded:
    """k_decode_window on USER16 slots: USER24's decode, the trace from a traced record's
    continuation slot, continuation slots holes (ts 0, no slot, no keys)."""
    v, cont = records.user16_to_user24(u)
    d = decode_user24(v, pod_sn, base)
    for f, z in (("ts", 0), ("val", 0), ("slot", NO_SLOT), ("status", 0), ("pod", 0), ("pid", 0), ("svcnode", 0),
                 ("trace", 0), ("conn", 0)):
        getattr(d, f)[cont] = z
    return d


def decode_window(framed: np.ndarray, user: np.ndarray, table: CtxTable, tmap: TraceMap, bases,
                  pod_sn: Dict[int, int] = None) -> Decoded:
    """k_decode_window: rows [0, n framed) from the slots of the framed batch records (row r =
    slot r % 8 of record r // 8; definitions, pads, discarded and busy records are holes: ts 0,
    no slot; kernel trace ids become their hashes), then the user-space records (trace hashes
    as is, conn32 connections)."""
    hdr, sl = records.framed_slots(framed)
    n_k = sl.shape[0]
    ev = sl.copy().view(records.EVENT16).reshape(-1)
    valid = (hdr == records.REC_PAYLOAD) & ((ev["ctx_type"] & np.uint32(0xFF)) < records.DEF_FIRST)
    d = decode_w16(ev, table, bases)
    d.trace = tmap.hashes(d.trace)
    if pod_sn:  # the pod's service as the pod table knows it now (not when its context was defined)
        now = np.array([pod_sn.get(int(p), 0) for p in d.pod.tolist()], dtype=np.uint32)
        d.svcnode = np.where(now != 0, now, d.svcnode).astype(d.svcnode.dtype)
    hole = ~valid
    for f, z in (("ts", 0), ("val", 0), ("slot", NO_SLOT), ("status", 0), ("pod", 0), ("pid", 0), ("svcnode", 0),
                 ("trace", 0), ("conn", 0)):
        getattr(d, f)[hole] = z
    if not len(user):
        return d
    if user.dtype == records.USER32:
        u = decode_user32(user, pod_sn or {})
    elif user.dtype == records.USER24:
        u = decode_user24(user, pod_sn or {}, max(int(b) for b in bases))
    elif user.dtype == records.USER16:
        u = decode_user16(user, pod_sn or {}, max(int(b) for b in bases))
    else:
        u = decode_events(user)
        u.conn = records.conn32_np(u.conn).astype(np.uint64)
    cat = lambda a, b: np.concatenate([a, b])  # noqa: E731
    assert n_k == len(d.ts)
    return Decoded(cat(d.ts, u.ts), cat(d.val, u.val), cat(d.slot, u.slot), cat(d.status, u.status), cat(d.pod, u.pod),
                   cat(d.pid, u.pid), cat(d.svcnode, u.svcnode), cat(d.trace, u.trace), cat(d.conn, u.conn))


def spans_native(spans: np.ndarray, tmap: TraceMap = None) -> np.ndarray:
    """k_decode_spans in the native engine: trace hashes as is, connections as conn32."""
    out = spans.copy()
    out["conn_h"] = records.conn32_np(spans["conn_h"])
    return out


# ---- imported rows (ops/csrc/exchange.hip) ----------------------------------------------

def concat(a: Decoded, b: Decoded) -> Decoded:
    return Decoded(*(np.concatenate([getattr(a, f), getattr(b, f)]) for f in Decoded.__dataclass_fields__))


def take(d: Decoded, m: np.ndarray) -> Decoded:
    return Decoded(*(getattr(d, f)[m] for f in Decoded.__dataclass_fields__))


def empty_rows() -> Decoded:
    return Decoded(np.zeros(0, np.int64), np.zeros(0, np.float32), np.zeros(0, np.uint8), np.zeros(0, np.uint8),
                   np.zeros(0, np.uint32), np.zeros(0, np.uint32), np.zeros(0, np.uint32), np.zeros(0, np.uint64),
                   np.zeros(0, np.uint64))


def window_tmax(d: Decoded, n_local: int) -> int:
    """Latest timestamp of the window's own joinable records (k_decode_window's tmax)."""
    ts = d.ts[:n_local]
    ok = (d.slot[:n_local] != NO_SLOT) & (ts > 0)
    return int(ts[ok].max()) if ok.any() else 0


def halo_rows(d: Decoded, n_local: int, halo_ns: int) -> Decoded:
    """k_sel (halo): the window's rows (imports included) within halo_ns of its latest local
    record, in row order."""
    tmax = window_tmax(d, n_local)
    if tmax == 0:
        return empty_rows()
    m = (d.slot != NO_SLOT) & (d.ts != 0) & (d.ts >= tmax - halo_ns)
    return take(d, m)


def trace_rows(d: Decoded, n_local: int) -> Decoded:
    """k_sel (trace): the window's own trace-tagged joinable rows at warn level or above,
    identity cleared (a remote GPU joins them by trace hash only), in row order."""
    loc = take(d, np.arange(len(d.ts)) < n_local)
    m = (loc.slot != NO_SLOT) & (loc.ts != 0) & (loc.trace != 0) & (loc.status >= 1)
    out = take(loc, m)
    for f in ("pod", "pid", "svcnode"):
        setattr(out, f, np.zeros_like(getattr(out, f)))
    out.conn = np.zeros_like(out.conn)
    return out


def status_of(val: np.ndarray, slot: np.ndarray) -> np.ndarray:
    warn = np.array([s.warn for s in catalog.SIGNALS] + [np.inf] * (16 - len(catalog.SIGNALS)), dtype=np.float32)
    err = np.array([s.error for s in catalog.SIGNALS] + [np.inf] * (16 - len(catalog.SIGNALS)), dtype=np.float32)
    ok = slot != NO_SLOT
    sl = np.where(ok, slot, 0)
    return np.where(ok, np.where(val >= err[sl], 2, np.where(val >= warn[sl], 1, 0)), 0).astype(np.uint8)


SIGREC = np.dtype([("ts", "<i8"), ("tr", "<u8"), ("cn", "<u8"), ("pod", "<u4"), ("pid", "<u4"), ("sn", "<u4"),
                   ("val", "<f4"), ("slot", "<u4"), ("pad", "<u4", (5,))])
assert SIGREC.itemsize == 64


def to_sigrec(d: Decoded) -> np.ndarray:
    """Decoded rows as the engine's 64-byte SigRec rows (mislo_common.h)."""
    out = np.zeros(len(d.ts), dtype=SIGREC)
    out["ts"], out["tr"], out["cn"] = d.ts, d.trace, d.conn
    out["pod"], out["pid"], out["sn"] = d.pod, d.pid, d.svcnode
    out["val"] = d.val
    out["slot"] = np.where(d.slot == NO_SLOT, 0xFF, d.slot).astype(np.uint32)
    return out


def from_sigrec(r: np.ndarray) -> Decoded:
    slot = np.where(r["slot"] == 0xFF, NO_SLOT, r["slot"]).astype(np.uint8)
    return Decoded(r["ts"].astype(np.int64), r["val"].astype(np.float32), slot, status_of(r["val"], slot),
                   r["pod"].astype(np.uint32), r["pid"].astype(np.uint32), r["sn"].astype(np.uint32),
                   r["tr"].astype(np.uint64), r["cn"].astype(np.uint64))


XREC = np.dtype([("ts", "<i8"), ("tr", "<u8"), ("val", "<f4"), ("slot", "<u4")])
assert XREC.itemsize == 24


def exchange_blocks(parts, cap: int) -> np.ndarray:
    """Per-rank exchange blocks as the GPUs all-gather them (mislo_launch.h XRec):
    [24-byte header: row count | 24-byte rows]."""
    stride = XREC.itemsize * (1 + cap)
    out = np.zeros(len(parts) * stride, dtype=np.uint8)
    for r, p in enumerate(parts):
        n = min(len(p.ts), cap)
        rows = np.zeros(n, dtype=XREC)
        rows["ts"], rows["tr"], rows["val"] = p.ts[:n], p.trace[:n], p.val[:n]
        rows["slot"] = np.where(p.slot[:n] == NO_SLOT, 0xFF, p.slot[:n])
        blk = out[r * stride:(r + 1) * stride]
        blk[:4] = np.frombuffer(np.uint32(n).tobytes(), dtype=np.uint8)
        blk[XREC.itemsize:XREC.itemsize + rows.nbytes] = rows.view(np.uint8)
    return out


def remote_rows(p: Decoded) -> Decoded:
    """What a GPU imports from an exchanged row: time, trace hash, value, signal; no identity."""
    z32 = np.zeros(len(p.ts), np.uint32)
    return Decoded(p.ts.copy(), p.val.copy(), p.slot.copy(), status_of(p.val, p.slot), z32, z32.copy(), z32.copy(),
                   p.trace.copy(), np.zeros(len(p.ts), np.uint64))


def decode_span20(sp: np.ndarray, table: CtxTable) -> np.ndarray:
    """k_decode_spans on SPAN20 records, as 64-byte SPAN records for ``join``."""
    row = table.rows(sp["ctx_id"].astype(np.int64))
    out = np.zeros(sp.shape[0], dtype=records.SPAN)
    out["ts_ns"] = sp["ts_ns"]
    out["trace_h"] = sp["trace_id"]
    out["conn_h"] = row[:, 2]
    out["pod_id"] = row[:, 0]
    out["pid"] = row[:, 1]
    out["svc_id"] = (row[:, 3] >> np.uint32(16)).astype(np.uint16)
    out["node_id"] = (row[:, 3] & np.uint32(0xFFFF)).astype(np.uint16)
    out["group_id"] = sp["group_id"]
    return out


def histograms(d: Decoded) -> np.ndarray:
    edges = np.array([list(s.buckets) for s in catalog.SIGNALS], dtype=np.float32)
    h = np.zeros((16, 16), dtype=np.int64)
    for s in range(16):
        v = d.val[d.slot == s]
        b = (v[:, None] > edges[s][None, :15]).sum(axis=1)
        np.add.at(h[s], b, 1)
    return h


def milli_units(v) -> np.ndarray:
    """Fixed-point image used by the kernels for sums (mislo_common.h milli_units)."""
    m = np.rint(np.asarray(v, dtype=np.float32).astype(np.float64) * 1000.0)
    return np.where(m > 0, m, 0).astype(np.int64)


def group_features(gsum: np.ndarray, gcnt: np.ndarray) -> np.ndarray:
    """k_group_features: float((gsum * 1e-3) / gcnt) in double, NaN where no pairs."""
    with np.errstate(invalid="ignore", divide="ignore"):
        return np.where(gcnt > 0, (gsum.astype(np.float64) * 1e-3) / np.maximum(gcnt, 1), np.nan).astype(np.float32)


def value_sums_milli(d: Decoded) -> np.ndarray:
    """Per-slot exact integer sums of rint(val * 1000) (decode kernels' misc[2:18])."""
    out = np.zeros(16, dtype=np.int64)
    ok = d.slot != NO_SLOT
    milli = np.rint(d.val[ok].astype(np.float64) * 1000.0)
    milli = np.where(milli > 0, milli, 0).astype(np.int64)
    np.add.at(out, d.slot[ok].astype(np.int64), milli)
    return out


@dataclass
class JoinResult:
    top3: np.ndarray        # uint64 [S,3]
    cnt: np.ndarray         # [S]
    attrs: np.ndarray       # float32 [S,16]
    conf: np.ndarray        # float32 [S]
    gsum: np.ndarray        # int64 [G,16] sums of milli-unit values (exact, order-free)
    gcnt: np.ndarray        # int64 [G,16]
    feat: np.ndarray        # float32 [G,16]
    debug: Dict[str, int]


class _KeyIndex:
    """Valid rows grouped by one join key, each group's rows sorted by time: the rows of a key
    within [t - w, t + w] are one contiguous slice (two binary searches)."""

    def __init__(self, keys: np.ndarray, ts: np.ndarray, rows: np.ndarray):
        if len(rows) == 0:
            self.groups, self.starts, self.ts, self.rows = {}, np.zeros(1, np.int64), ts[:0], rows[:0]
            return
        uniq, inv = np.unique(keys, axis=0, return_inverse=True)
        inv = inv.reshape(-1)
        order = np.lexsort((ts, inv))
        self.ts, self.rows = ts[order], rows[order]
        self.starts = np.concatenate([[0], np.cumsum(np.bincount(inv, minlength=len(uniq)))]).astype(np.int64)
        self.groups = {tuple(int(x) for x in np.atleast_1d(u)): i for i, u in enumerate(uniq)}

    def near(self, key: tuple, t: int, w: int) -> np.ndarray:
        g = self.groups.get(key)
        if g is None:
            return self.rows[:0]
        lo, hi = int(self.starts[g]), int(self.starts[g + 1])
        seg = self.ts[lo:hi]
        a = lo + int(np.searchsorted(seg, t - w, side="left"))
        b = lo + int(np.searchsorted(seg, t + w, side="right"))
        return self.rows[a:b]


def join(d: Decoded, spans: np.ndarray, n_groups: int, window_ms: float = 2000.0, threshold: float = 0.7,
         fanout: int = 3, group_mode: int = 1) -> JoinResult:
    """The REF 4-tier join of every span with the window's rows, exactly ``join_bruteforce``'s
    result: a row is a candidate of a span only through one of the tiers' key equalities, so
    each span looks at the union of its trace / (pod, pid) / (pod, conn) / (svc, node) groups'
    rows within the tier's time reach (``_KeyIndex``) and applies the same per-row rules there.
    O(rows log rows + spans x reachable rows) instead of O(spans x rows): the headline window
    (1M rows x 16K spans) in minutes instead of hours."""
    outer = int(round(window_ms * MS))
    if outer <= 0:
        outer = 2000 * MS
    win = [outer, min(outer, 100 * MS), min(outer, 250 * MS), min(outer, 500 * MS)]
    thr = np.float32(threshold)
    confs = np.array(TIER_CONF, dtype=np.float32)
    S = spans.shape[0]
    N = d.ts.shape[0]
    supported = d.slot != NO_SLOT
    n_sup = int(supported.sum())
    top3 = np.full((S, 3), np.uint64(0xFFFFFFFFFFFFFFFF), dtype=np.uint64)
    cnt = np.zeros(S, dtype=np.int64)
    attrs = np.full((S, 16), np.nan, dtype=np.float32)
    conf = np.zeros(S, dtype=np.float32)
    gsum = np.zeros((n_groups, 16), dtype=np.int64)
    gcnt = np.zeros((n_groups, 16), dtype=np.int64)
    matched_total = low_total = dropped_total = 0
    sp_svcnode = (spans["svc_id"].astype(np.uint32) << np.uint32(16)) | spans["node_id"].astype(np.uint32)
    valid = supported & (d.ts != 0)
    vi = np.nonzero(valid)[0].astype(np.int64)
    vts = d.ts[vi]
    m1 = d.trace[vi] != 0
    m2 = (d.pod[vi] != 0) & (d.pid[vi] != 0)
    m3 = (d.pod[vi] != 0) & (d.conn[vi] != 0)
    sn_v = d.svcnode[vi]
    m4 = ((sn_v >> np.uint32(16)) != 0) & ((sn_v & np.uint32(0xFFFF)) != 0)
    ix_tr = _KeyIndex(d.trace[vi][m1].astype(np.uint64), vts[m1], vi[m1])
    ix_pp = _KeyIndex(np.stack([d.pod[vi][m2].astype(np.uint64), d.pid[vi][m2].astype(np.uint64)], 1), vts[m2], vi[m2])
    ix_pc = _KeyIndex(np.stack([d.pod[vi][m3].astype(np.uint64), d.conn[vi][m3]], 1), vts[m3], vi[m3])
    ix_sn = _KeyIndex(sn_v[m4].astype(np.uint64), vts[m4], vi[m4])
    for s in range(S):
        t = int(spans["ts_ns"][s])
        if t == 0:
            continue
        tr = int(spans["trace_h"][s])
        pod, pid, cn, sn = int(spans["pod_id"][s]), int(spans["pid"][s]), int(spans["conn_h"][s]), int(sp_svcnode[s])
        parts = []
        if tr:
            parts.append(ix_tr.near((tr,), t, win[0]))
        if pod and pid:
            parts.append(ix_pp.near((pod, pid), t, win[1]))
        if pod and cn:
            parts.append(ix_pc.near((pod, cn), t, win[2]))
        if (sn >> 16) and (sn & 0xFFFF):
            parts.append(ix_sn.near((sn,), t, win[3]))
        grp = int(spans["group_id"][s])
        rows = np.unique(np.concatenate(parts)) if parts else vi[:0]
        if rows.size:
            dt = np.abs(d.ts[rows] - t)
            outer_ok = dt <= outer
            t1 = outer_ok & (np.uint64(tr) != 0) & (d.trace[rows] == np.uint64(tr))
            t2 = outer_ok & (pod != 0) & (d.pod[rows] == np.uint32(pod)) & (pid != 0) & (d.pid[rows] == np.uint32(pid)) \
                & (dt <= win[1])
            t3 = outer_ok & (pod != 0) & (d.pod[rows] == np.uint32(pod)) & (cn != 0) & (d.conn[rows] == np.uint64(cn)) \
                & (dt <= win[2])
            t4 = outer_ok & ((sn >> 16) != 0) & ((sn & 0xFFFF) != 0) & (d.svcnode[rows] == np.uint32(sn)) & (dt <= win[3])
            tier = np.where(t1, 1, np.where(t2, 2, np.where(t3, 3, np.where(t4, 4, 0))))
            m = tier > 0
            c = np.zeros(rows.size, dtype=np.float32)
            c[m] = confs[tier[m] - 1]
            cand = m & (c >= thr)
            matched_total += int(m.sum())
            low_total += int((m & (c < thr)).sum())
            ci = rows[cand]
            cnt[s] = ci.size
            if ci.size:
                keys = ((tier[cand].astype(np.uint64) - np.uint64(1)) << np.uint64(62)) | \
                       (dt[cand].astype(np.uint64) << np.uint64(SIG_BITS)) | ci.astype(np.uint64)
                keys.sort()
                k3 = keys[:3]
                top3[s, :k3.size] = k3
                mc = np.float32(0)
                for key in keys[:min(fanout, 3)]:
                    g = int(key & np.uint64((1 << SIG_BITS) - 1))
                    sl = int(d.slot[g])
                    v = d.val[g]
                    if np.isnan(attrs[s, sl]) or v > attrs[s, sl]:
                        attrs[s, sl] = v
                    mc = max(mc, confs[int(key >> np.uint64(62))])
                conf[s] = mc
                dropped_total += max(0, ci.size - fanout)
                if group_mode == 1 and grp < n_groups:
                    np.add.at(gsum[grp], d.slot[ci].astype(np.int64), milli_units(d.val[ci]))
                    np.add.at(gcnt[grp], d.slot[ci].astype(np.int64), 1)
        if group_mode == 0 and grp < n_groups:
            p = ~np.isnan(attrs[s])
            gsum[grp][p] += milli_units(attrs[s][p])
            gcnt[grp][p] += 1
    with np.errstate(invalid="ignore", divide="ignore"):
        feat = group_features(gsum, gcnt)
    n_uns = N - n_sup
    debug = {
        "candidates": int(cnt.sum()), "low_confidence": low_total, "fanout_dropped": dropped_total,
        "unmatched": S * n_sup - matched_total, "unsupported_type": S * n_uns,
        "spans_enriched": int((conf > 0).sum()),
    }
    return JoinResult(top3, cnt, attrs, conf, gsum, gcnt, feat, debug)


def join_bruteforce(d: Decoded, spans: np.ndarray, n_groups: int, window_ms: float = 2000.0, threshold: float = 0.7,
                    fanout: int = 3, group_mode: int = 1) -> JoinResult:
    """Every span against every row: the literal statement of the join (``join`` is its indexed
    equivalent, checked against it in tests/test_oracle.py)."""
    outer = int(round(window_ms * MS))
    if outer <= 0:
        outer = 2000 * MS
    win = [outer, min(outer, 100 * MS), min(outer, 250 * MS), min(outer, 500 * MS)]
    thr = np.float32(threshold)
    confs = np.array(TIER_CONF, dtype=np.float32)
    S = spans.shape[0]
    N = d.ts.shape[0]
    supported = d.slot != NO_SLOT
    n_sup = int(supported.sum())
    idx_all = np.arange(N, dtype=np.uint64)
    top3 = np.full((S, 3), np.uint64(0xFFFFFFFFFFFFFFFF), dtype=np.uint64)
    cnt = np.zeros(S, dtype=np.int64)
    attrs = np.full((S, 16), np.nan, dtype=np.float32)
    conf = np.zeros(S, dtype=np.float32)
    gsum = np.zeros((n_groups, 16), dtype=np.int64)
    gcnt = np.zeros((n_groups, 16), dtype=np.int64)
    matched_total = low_total = dropped_total = 0
    sp_svcnode = (spans["svc_id"].astype(np.uint32) << np.uint32(16)) | spans["node_id"].astype(np.uint32)
    for s in range(S):
        t = int(spans["ts_ns"][s])
        if t == 0:
            continue
        valid = supported & (d.ts != 0)
        dt = np.abs(d.ts - t)
        outer_ok = valid & (dt <= outer)
        tr = np.uint64(spans["trace_h"][s])
        pod = np.uint32(spans["pod_id"][s])
        pid = np.uint32(spans["pid"][s])
        cn = np.uint64(spans["conn_h"][s])
        sn = sp_svcnode[s]
        t1 = outer_ok & (tr != 0) & (d.trace == tr)
        t2 = outer_ok & (pod != 0) & (d.pod == pod) & (pid != 0) & (d.pid == pid) & (dt <= win[1])
        t3 = outer_ok & (pod != 0) & (d.pod == pod) & (cn != 0) & (d.conn == cn) & (dt <= win[2])
        t4 = outer_ok & ((sn >> np.uint32(16)) != 0) & ((sn & np.uint32(0xFFFF)) != 0) & (d.svcnode == sn) & (dt <= win[3])
        tier = np.where(t1, 1, np.where(t2, 2, np.where(t3, 3, np.where(t4, 4, 0))))
        m = tier > 0
        c = np.zeros(N, dtype=np.float32)
        c[m] = confs[tier[m] - 1]
        cand = m & (c >= thr)
        low = m & (c < thr)
        matched_total += int(m.sum())
        low_total += int(low.sum())
        ci = np.nonzero(cand)[0]
        cnt[s] = ci.size
        if ci.size:
            keys = ((tier[ci].astype(np.uint64) - np.uint64(1)) << np.uint64(62)) | \
                   (dt[ci].astype(np.uint64) << np.uint64(SIG_BITS)) | idx_all[ci]
            keys.sort()
            k3 = keys[:3]
            top3[s, :k3.size] = k3
            keep = keys[:min(fanout, 3)]
            mc = np.float32(0)
            for key in keep:
                g = int(key & np.uint64((1 << SIG_BITS) - 1))
                sl = int(d.slot[g])
                v = d.val[g]
                if np.isnan(attrs[s, sl]) or v > attrs[s, sl]:
                    attrs[s, sl] = v
                mc = max(mc, confs[int(key >> np.uint64(62))])
            conf[s] = mc
            dropped_total += max(0, ci.size - fanout)
            grp = int(spans["group_id"][s])
            if group_mode == 1 and grp < n_groups:
                np.add.at(gsum[grp], d.slot[ci].astype(np.int64), milli_units(d.val[ci]))
                np.add.at(gcnt[grp], d.slot[ci].astype(np.int64), 1)
        grp = int(spans["group_id"][s])
        if group_mode == 0 and grp < n_groups:
            p = ~np.isnan(attrs[s])
            gsum[grp][p] += milli_units(attrs[s][p])
            gcnt[grp][p] += 1
    with np.errstate(invalid="ignore", divide="ignore"):
        feat = group_features(gsum, gcnt)
    n_uns = N - n_sup
    debug = {
        "candidates": int(cnt.sum()), "low_confidence": low_total, "fanout_dropped": dropped_total,
        "unmatched": S * n_sup - matched_total, "unsupported_type": S * n_uns,
        "spans_enriched": int((conf > 0).sum()),
    }
    return JoinResult(top3, cnt, attrs, conf, gsum, gcnt, feat, debug)
