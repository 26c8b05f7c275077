"""Binary event/span record formats shared by the BPF probes, the native ring and the GPU.

* ``REF_EVENT`` -- REF's packed 40-byte ``struct llm_slo_event``
  (ebpf/c/llm_slo_event.h:32-42). Accepted for replay compatibility; decoded with REF's
  exact rules (pkg/collector/ringbuf.go:152-243): type->(name, unit), count stays a count,
  cpu_steal stays raw ns, everything else ns/1e6 -> ms, conn tuple only if a port != 0
  (src_ip "0.0.0.0", protocol "tcp"), errno only if != 0, IPv4 little-endian bytes.
* ``EVENT`` -- NEW 64-byte, 64-byte-aligned record (one cache line per event, 16-B
  aligned fields for dwordx4 loads on gfx950). It keeps every REF field and adds
  interned workload ids (pod/node/service), a 64-bit trace-id hash, a 64-bit
  connection hash, a GPU id and flags. Layout is mirrored in
  ``ops/csrc/mislo_records.h`` and ``ebpf/c/mislo_event.h``.
* ``SPAN`` -- 64-byte span record for the correlation join.
"""

from __future__ import annotations

import numpy as np

from ..contracts.types import ConnTuple, ProbeEventV1
from ..signals import catalog

REF_EVENT = np.dtype([
    ("pid", "<u4"), ("tid", "<u4"), ("timestamp_ns", "<u8"), ("signal_type", "<u4"),
    ("value_ns", "<u8"), ("conn_src_port", "<u2"), ("conn_dst_port", "<u2"),
    ("conn_dst_ip", "<u4"), ("errno_val", "<i4"),
], align=False)
assert REF_EVENT.itemsize == 40

EVENT = np.dtype([
    ("ts_ns", "<i8"),        # 0   CLOCK_REALTIME ns (probes convert ktime at the boundary)
    ("value", "<u8"),        # 8   raw value in the signal's kernel unit (see catalog.decode_scale)
    ("trace_h", "<u8"),      # 16  64-bit trace-id hash, 0 = none
    ("pid", "<u4"),          # 24
    ("tid", "<u4"),          # 28
    ("pod_id", "<u4"),       # 32  interned pod id, 0 = unknown
    ("dst_ip", "<u4"),       # 36  IPv4 (network order as read by the probe)
    ("signal_type", "<u2"),  # 40
    ("node_id", "<u2"),      # 42  interned node id
    ("svc_id", "<u2"),       # 44  interned service id
    ("flags", "<u2"),        # 46  bits 0-7 gpu id, bit 8 has_gpu, bit 9 synthetic
    ("src_port", "<u2"),     # 48
    ("dst_port", "<u2"),     # 50
    ("errno", "<i4"),        # 52
    ("conn_h", "<u8"),       # 56  connection hash (0 -> derived on device from ports/ip)
])
assert EVENT.itemsize == 64

EVENT32 = np.dtype([
    ("ts_ns", "<i8"),        # 0
    ("trace_h", "<u8"),      # 8
    ("value_milli", "<u4"),  # 16 value in 1/1000 of the signal's output unit
    ("pid", "<u4"),          # 20
    ("pod_id", "<u4"),       # 24 interned pod id (svc/node via the device pod table)
    ("type_conn", "<u4"),    # 28 bits 0-7 signal_type, bits 8-31 interned connection id
])
assert EVENT32.itemsize == 32

# 20-byte wire record: the window's base timestamp travels once per window (counts[4..5]),
# pod / pid / connection / svc|node travel once per distinct context (the device context
# table, CtxInterner); only the trace hash stays per event. 5/8 of EVENT32's PCIe bytes.
EVENT20 = np.dtype({"names": ["ts_off", "ctx_type", "value_milli", "trace_h"],
                    "formats": ["<u4", "<u4", "<u4", "<u8"],
                    "offsets": [0, 4, 8, 12], "itemsize": 20})
TS_ZERO = 0xFFFFFFFF  # ts_off of a zero timestamp (never joins)
assert EVENT20.itemsize == 20

# 16-byte record (= probes/ebpf/mislo_record.h mislo_event16 with -DMISLO_RING_EVENT16, or the
# host encoding): EVENT20 with the trace hash interned to a 30-bit id shared with the window's
# spans (TraceInterner / the native WireEncoder / the kernel's mislo_traces), and a 2-bit epoch
# tag: ts = base[tag] + ts_off, the window carrying its last 4 epoch bases (counts[4..5],
# counts[8..13]). The host encoder writes tag 0 (one base per window).
EVENT16 = np.dtype([
    ("ts_off", "<u4"),       # 0  ns since the tagged epoch base, TS_ZERO = zero timestamp
    ("ctx_type", "<u4"),     # 4  bits 0-7 signal type, 8-31 context id
    ("value_milli", "<u4"),  # 8
    ("trace_id", "<u4"),     # 12 bits 0-29 interned trace id (0 = none), 30-31 epoch tag
])
EPOCH_TAG_SHIFT = 30
TRACE_ID_MASK = (1 << EPOCH_TAG_SHIFT) - 1
COUNTS_LEN = 16  # per-window counts int32[16]: sizes, epoch bases, context rows (ops/csrc)


class EpochClock:
    """The agent's half of the EVENT16 epoch protocol (probes/ebpf/mislo_probe.h). At each window
    cut the agent publishes epoch k into mislo_cfg[MISLO_CFG_EPOCH] as ``base | (k & 3)`` (base =
    realtime ns rounded down to a multiple of 4) and remembers the base under tag k & 3. A probe
    stamps ``ts - base`` with the tag of the epoch it read, so a record written across a cut
    still names its own base; the window ships the last 4 bases (``counts_row(bases=...)``),
    indexed by tag, and decodes records stamped up to 3 cuts late exactly."""

    def __init__(self):
        self.k = -1
        self._bases = [0, 0, 0, 0]

    def publish(self, now_ns: int) -> int:
        """Start epoch k+1 at ``now_ns``; returns the mislo_cfg value to write."""
        self.k += 1
        base = int(now_ns) & ~3
        self._bases[self.k & 3] = base
        return base | (self.k & 3)

    def bases(self) -> tuple:
        """Epoch bases indexed by tag (counts[4..5], [8..13])."""
        return tuple(self._bases)

    @staticmethod
    def stamp(ts_ns: int, cfg_value: int) -> tuple:
        """(ts_off, tag) exactly as mislo_submit computes them from a cfg value it read."""
        base, tag = int(cfg_value) & ~3, int(cfg_value) & 3
        if ts_ns == 0:
            return TS_ZERO, tag
        if ts_ns < base:
            return 0, tag
        d = ts_ns - base
        return (TS_ZERO - 1 if d >= TS_ZERO else d), tag


def retag_epochs(ev16: np.ndarray, t_base: int, period_ns: int):
    """Re-express EVENT16 records (tag 0, offsets from ``t_base``) the way probes stamp them when
    the agent publishes a new epoch every ``period_ns`` inside the window: epoch j = t_base +
    j * period_ns (j <= 3), each record offset from the latest epoch at or before it, with tag j.
    Returns (records, bases); decoding with ``bases`` gives back the same timestamps."""
    out = ev16.copy()
    off = ev16["ts_off"].astype(np.int64)
    live = off != TS_ZERO
    j = np.where(live, np.minimum(off // int(period_ns), 3), 0).astype(np.int64)
    out["ts_off"] = np.where(live, off - j * int(period_ns), TS_ZERO).astype(np.uint32)
    out["trace_id"] = (ev16["trace_id"].astype(np.uint32) & np.uint32(TRACE_ID_MASK)) | \
        (j.astype(np.uint32) << np.uint32(EPOCH_TAG_SHIFT))
    return out, tuple(int(t_base) + k * int(period_ns) for k in range(4))


def counts_row(n_ev: int, n_sp: int, n_groups: int, n_local: int = 0, bases=(0,), n_ctx: int = 0,
               span_bytes: int = 64) -> np.ndarray:
    """The window's counts int32[16] as the decode kernels read them: [0] events, [1] spans,
    [2] incident groups, [3] node-local events (0 = all), [4..5] epoch base 0 (the window base),
    [6] valid context rows, [7] span record bytes (20 = SPAN20, else 64-byte SPAN),
    [8..9] / [10..11] / [12..13] epoch bases 1-3 (EVENT16 tags)."""
    b = [int(x) & 0xFFFFFFFFFFFFFFFF for x in (list(bases) + [0, 0, 0, 0])[:4]]
    v = [n_ev, n_sp, n_groups, n_local, b[0] & 0xFFFFFFFF, b[0] >> 32, n_ctx, 20 if span_bytes == 20 else 0,
         b[1] & 0xFFFFFFFF, b[1] >> 32, b[2] & 0xFFFFFFFF, b[2] >> 32, b[3] & 0xFFFFFFFF, b[3] >> 32, 0, 0]
    return np.array(v, dtype=np.uint64).astype(np.uint32).view(np.int32)
assert EVENT16.itemsize == 16
# 24-byte record (= probes/ebpf/mislo_record.h mislo_event24): what the probes put on the
# ring when the kernel interns the workload context too: absolute timestamp (no window base
# at the source), trace hash, fixed-point value, context id into the device context table.
EVENT24 = np.dtype([
    ("ts_ns", "<i8"),        # 0
    ("trace_h", "<u8"),      # 8
    ("value_milli", "<u4"),  # 16
    ("ctx_type", "<u4"),     # 20 bits 0-7 signal type, 8-31 context id
])
assert EVENT24.itemsize == 24
# 20-byte record (= probes/ebpf/mislo_record.h mislo_event20t, the probes' default ring
# record): EVENT24 with the trace hash interned in the kernel to a 32-bit id (mislo_traces);
# the agent puts the window's spans on the same ids. Records sit at 20-byte strides. Its wire
# code is 21 (20 is EVENT20, the window-relative host encoding): see wire_bytes().
EVENT20T = np.dtype({"names": ["ts_ns", "value_milli", "ctx_type", "trace_id"],
                     "formats": ["<i8", "<u4", "<u4", "<u4"],
                     "offsets": [0, 8, 12, 16], "itemsize": 20})
assert EVENT20T.itemsize == 20
WIRE_20T = 21
WIRE_DTYPES = {64: EVENT, 32: EVENT32, 24: EVENT24, WIRE_20T: EVENT20T, 20: EVENT20, 16: EVENT16}
# bench / agent spelling of the wire codes
WIRE_NAMES = {"64": 64, "32": 32, "24": 24, "20t": WIRE_20T, "20": 20, "16": 16, "16t": 16}  # 16t: EVENT16 ring


def wire_bytes(wire: int) -> int:
    """PCIe bytes per event of wire code ``wire`` (21 = EVENT20T is 20 bytes)."""
    return 20 if wire == WIRE_20T else int(wire)


def wire_code(dtype: np.dtype) -> int:
    """Wire code of a record dtype (itemsize, except EVENT20T -> 21)."""
    for code, dt in WIRE_DTYPES.items():
        if dt == dtype:
            return code
    raise TypeError(f"not a wire record dtype: {dtype}")

SPAN = np.dtype([
    ("ts_ns", "<i8"),        # 0
    ("trace_h", "<u8"),      # 8
    ("conn_h", "<u8"),       # 16
    ("pid", "<u4"),          # 24
    ("pod_id", "<u4"),       # 28
    ("node_id", "<u2"),      # 32
    ("svc_id", "<u2"),       # 34
    ("group_id", "<u4"),     # 36 incident group (service x window) for aggregation
    ("ttft_ms", "<f4"),      # 40
    ("latency_ms", "<f4"),   # 44
    ("span_h", "<u8"),       # 48
    ("reserved", "<u8"),     # 56
])
assert SPAN.itemsize == 64

FLAG_HAS_GPU = 1 << 8
FLAG_SYNTHETIC = 1 << 9

# REF kernel type ids (ringbuf.go:29-39)
REF_TYPE_CPU_STEAL = 6
REF_TYPE_TCP_RETRANSMIT = 2


def ipv4_from_u32(ip: int) -> str:
    """REF ipFromU32 (ringbuf.go:240-243): little-endian byte order."""
    ip = int(ip)
    return f"{ip & 0xFF}.{(ip >> 8) & 0xFF}.{(ip >> 16) & 0xFF}.{(ip >> 24) & 0xFF}"


def ref_convert_value(signal_type: int, value_ns: int) -> float:
    """REF convertValue (ringbuf.go:229-238)."""
    if signal_type in (REF_TYPE_TCP_RETRANSMIT, REF_TYPE_CPU_STEAL):
        return float(value_ns)
    return float(value_ns) / 1e6


def ref_signal_from_type(signal_type: int):
    """REF signalFromType (ringbuf.go:199-225): cpu_steal unit is "ns" at the kernel boundary."""
    if signal_type == REF_TYPE_CPU_STEAL:
        return "cpu_steal_pct", "ns"
    if 1 <= signal_type <= 9:
        return catalog.signal_from_type(signal_type)
    return "unknown", "unknown"


def decode_ref_record(buf: bytes, meta, ts_unix_nano: int) -> ProbeEventV1:
    """Decode one 40-byte REF record exactly like REF toProbeEvent (ringbuf.go:161-197).

    ``meta`` supplies node/namespace/pod/container/trace_id/span_id (EventMetadata);
    REF stamps wall-clock ``time.Now()`` -- the caller passes it as ``ts_unix_nano``.
    """
    if len(buf) < REF_EVENT.itemsize:
        raise ValueError("decode bpf event: short buffer")
    r = np.frombuffer(buf[: REF_EVENT.itemsize], dtype=REF_EVENT)[0]
    st = int(r["signal_type"])
    name, unit = ref_signal_from_type(st)
    ev = ProbeEventV1(
        ts_unix_nano=int(ts_unix_nano), signal=name, node=meta.node, namespace=meta.namespace,
        pod=meta.pod, container=meta.container, pid=int(r["pid"]), tid=int(r["tid"]),
        value=ref_convert_value(st, int(r["value_ns"])), unit=unit, status="ok",
        trace_id=meta.trace_id, span_id=meta.span_id)
    sp, dp = int(r["conn_src_port"]), int(r["conn_dst_port"])
    if sp != 0 or dp != 0:
        ev.conn_tuple = ConnTuple("0.0.0.0", ipv4_from_u32(int(r["conn_dst_ip"])), sp, dp, "tcp")
    if int(r["errno_val"]) != 0:
        ev.errno = int(r["errno_val"])
    return ev


def encode_ref_record(pid, tid, ts_ns, signal_type, value_ns, sport=0, dport=0, dst_ip=0, errno=0) -> bytes:
    a = np.zeros(1, dtype=REF_EVENT)
    a[0] = (pid, tid, ts_ns, signal_type, value_ns, sport, dport, dst_ip, errno)
    return a.tobytes()


DECODE_SCALE = np.array([s.decode_scale for s in catalog.SIGNALS], dtype=np.float64)


def type_to_slot_table(max_type: int = 128) -> np.ndarray:
    """signal_type -> slot (or -1). Kernel-side constant table."""
    t = np.full(max_type, -1, dtype=np.int32)
    for spec in catalog.SIGNALS:
        t[spec.kernel_type] = spec.slot
    return t


def conn_hash(src_port: int, dst_port: int, dst_ip: int) -> int:
    """64-bit connection hash (splitmix64 over the packed tuple). 0 when no port is set
    (REF builds a conn tuple only when a port != 0, ringbuf.go:181)."""
    if src_port == 0 and dst_port == 0:
        return 0
    x = ((int(src_port) & 0xFFFF) << 48) | ((int(dst_port) & 0xFFFF) << 32) | (int(dst_ip) & 0xFFFFFFFF)
    return splitmix64(x) or 1


def splitmix64(x: int) -> int:
    M = (1 << 64) - 1
    x = (x + 0x9E3779B97F4A7C15) & M
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    return z ^ (z >> 31)


def splitmix64_np(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def conn_hash_np(src_port: np.ndarray, dst_port: np.ndarray, dst_ip: np.ndarray) -> np.ndarray:
    sp = src_port.astype(np.uint64)
    dp = dst_port.astype(np.uint64)
    ip = dst_ip.astype(np.uint64)
    packed = (sp << np.uint64(48)) | (dp << np.uint64(32)) | ip
    h = splitmix64_np(packed)
    h = np.where(h == 0, np.uint64(1), h)
    return np.where((sp == 0) & (dp == 0), np.uint64(0), h)


def pod_table(events: np.ndarray, spans: np.ndarray = None) -> np.ndarray:
    """pod_id -> (svc << 16 | node) lookup table (int32) from records that carry both."""
    pods = [events["pod_id"]]
    sn = [(events["svc_id"].astype(np.uint32) << np.uint32(16)) | events["node_id"].astype(np.uint32)]
    if spans is not None and len(spans):
        pods.append(spans["pod_id"])
        sn.append((spans["svc_id"].astype(np.uint32) << np.uint32(16)) | spans["node_id"].astype(np.uint32))
    p = np.concatenate(pods).astype(np.int64)
    v = np.concatenate(sn)
    table = np.zeros(int(p.max()) + 1 if p.size else 1, dtype=np.uint32)
    table[p] = v
    return table.view(np.int32)


class ConnInterner:
    """64-bit connection hash -> dense 24-bit connection id (0 = no connection); the
    user-space side of the BPF probes' 5-tuple -> id map."""

    def __init__(self):
        self._ids = {}

    def ids(self, conn_h: np.ndarray) -> np.ndarray:
        uniq, inv = np.unique(conn_h, return_inverse=True)
        out = np.zeros(uniq.shape[0], dtype=np.uint32)
        for j, h in enumerate(uniq.tolist()):
            if h == 0:
                continue
            i = self._ids.get(h)
            if i is None:
                i = len(self._ids) + 1
                if i >= (1 << 24):
                    raise OverflowError("connection id space exhausted")
                self._ids[h] = i
            out[j] = i
        return out[inv]


def milli_shift_table() -> np.ndarray:
    """Per kernel signal type (< 256): the power of ten d with value_milli = raw * 10**d, i.e.
    log10(decode_scale * 1000). Every catalogue scale is a power of ten (ns -> ms: -3,
    counts: +3, milli-percent / ns -> us: 0), so the fixed-point conversion is integer-only
    and the BPF probes compute it in the kernel (probes/ebpf/mislo_record.h mislo_milli)."""
    shift = np.full(256, 3, dtype=np.int8)  # unknown types: scale 1
    for s in catalog.SIGNALS:
        if s.kernel_type < 256:
            d = float(np.log10(s.decode_scale * 1000.0))
            if abs(d - round(d)) > 1e-9 or not -9 <= round(d) <= 9:
                raise ValueError(f"{s.name}: decode_scale {s.decode_scale} is not a power of ten")
            shift[s.kernel_type] = int(round(d))
    return shift


def milli_int(raw: np.ndarray, shift: np.ndarray) -> np.ndarray:
    """raw * 10**shift rounded half-to-even, saturated to u32 (integer arithmetic only)."""
    v = raw.astype(np.uint64)
    d = shift.astype(np.int64)
    out = np.zeros(v.shape, dtype=np.uint64)
    lim = np.uint64(0xFFFFFFFF)
    for k in np.unique(d).tolist():
        m = d == k
        x = v[m]
        if k >= 0:
            p = np.uint64(10 ** k)
            big = x > lim // p if k else np.zeros(x.shape, bool)
            out[m] = np.where(big, lim, np.minimum(x * p, lim))
        else:
            p = np.uint64(10 ** (-k))
            q, r = x // p, x % p
            half = p // np.uint64(2)
            up = (r > half) | ((r == half) & ((q & np.uint64(1)) == np.uint64(1)))
            out[m] = np.minimum(q + up.astype(np.uint64), lim)
    return out.astype(np.uint32)


_SHIFT = None


def _milli_values(events: np.ndarray) -> np.ndarray:
    """Raw record values -> u32 thousandths of the signal's output unit (milli_int rule)."""
    global _SHIFT
    if _SHIFT is None:
        _SHIFT = milli_shift_table()
    st = events["signal_type"].astype(np.int64)
    shift = np.where(st < 256, _SHIFT[np.minimum(st, 255)], np.int8(3))
    return milli_int(events["value"], shift)


def _conn_keys(events: np.ndarray) -> np.ndarray:
    conn = events["conn_h"].copy()
    derived = conn_hash_np(events["src_port"], events["dst_port"], events["dst_ip"])
    return np.where(conn == 0, derived, conn)


def to_compact(events: np.ndarray, interner: "ConnInterner") -> np.ndarray:
    """EVENT (64 B) -> EVENT32 (32 B): milli-unit fixed point values, interned conn ids."""
    out = np.zeros(events.shape[0], dtype=EVENT32)
    out["ts_ns"] = events["ts_ns"]
    out["trace_h"] = events["trace_h"]
    out["value_milli"] = _milli_values(events)
    out["pid"] = events["pid"]
    out["pod_id"] = events["pod_id"]
    cid = interner.ids(_conn_keys(events))
    st = events["signal_type"].astype(np.uint32)
    out["type_conn"] = (st & np.uint32(0xFF)) | (cid << np.uint32(8))
    return out


def to_wire20(events: np.ndarray, conns: "ConnInterner", ctxs: "CtxInterner"):
    """EVENT (64 B) -> (EVENT20 (20 B), t_base): timestamps relative to the window's
    earliest non-zero timestamp, interned (pod, pid, conn, svc|node) contexts. Raises
    ValueError when the window spans 2^32 - 1 ns or more (use EVENT32 then)."""
    out = np.zeros(events.shape[0], dtype=EVENT20)
    ts = events["ts_ns"].astype(np.int64)
    nz = ts != 0
    t_base = int(ts[nz].min()) if nz.any() else 0
    off = ts - t_base
    if nz.any() and int(off[nz].max()) >= TS_ZERO:
        raise ValueError("window spans >= 2^32 ns: not representable in EVENT20")
    out["ts_off"] = np.where(nz, off, TS_ZERO).astype(np.uint32)
    out["value_milli"] = _milli_values(events)
    out["trace_h"] = events["trace_h"]
    cid = conns.ids(_conn_keys(events))
    sn = (events["svc_id"].astype(np.uint32) << np.uint32(16)) | events["node_id"].astype(np.uint32)
    ctx = ctxs.ids(events["pod_id"], events["pid"], cid, sn)
    st = events["signal_type"].astype(np.uint32)
    out["ctx_type"] = (st & np.uint32(0xFF)) | (ctx << np.uint32(8))
    return out, t_base


def to_wire24(events: np.ndarray, conns: "ConnInterner", ctxs: "CtxInterner") -> np.ndarray:
    """EVENT (64 B) -> EVENT24 (24 B), the probes' context-interned ring record: absolute
    timestamps, trace hash, fixed-point value, interned (pod, pid, conn, svc|node) context."""
    out = np.zeros(events.shape[0], dtype=EVENT24)
    out["ts_ns"] = events["ts_ns"]
    out["trace_h"] = events["trace_h"]
    out["value_milli"] = _milli_values(events)
    cid = conns.ids(_conn_keys(events))
    sn = (events["svc_id"].astype(np.uint32) << np.uint32(16)) | events["node_id"].astype(np.uint32)
    ctx = ctxs.ids(events["pod_id"], events["pid"], cid, sn)
    st = events["signal_type"].astype(np.uint32)
    out["ctx_type"] = (st & np.uint32(0xFF)) | (ctx << np.uint32(8))
    return out


def to_wire20t(events: np.ndarray, conns: "ConnInterner", ctxs: "CtxInterner",
               traces: "TraceInterner") -> np.ndarray:
    """EVENT (64 B) -> EVENT20T (20 B), the probes' default ring record: EVENT24 with the
    trace hash interned (spans must go through ``wire_spans`` with the same interners)."""
    e24 = to_wire24(events, conns, ctxs)
    out = np.zeros(events.shape[0], dtype=EVENT20T)
    for f in ("ts_ns", "value_milli", "ctx_type"):
        out[f] = e24[f]
    out["trace_id"] = traces.ids(events["trace_h"])
    return out


# 20-byte span record (ops/csrc SpanC20, runtime/csrc/wire.h Span20): what the GPU join reads of
# a span, with (pod, pid, conn, svc|node) as a context id and an interned trace id; used with the
# trace-interning event rings (EVENT16 / EVENT20T), 5/16 of the 64-byte SPAN's PCIe bytes.
SPAN20 = np.dtype({"names": ["ts_ns", "trace_id", "ctx_id", "group_id"],
                   "formats": ["<i8", "<u4", "<u4", "<u4"], "offsets": [0, 8, 12, 16], "itemsize": 20})


def to_span20(spans: np.ndarray, conns: "ConnInterner", ctxs: "CtxInterner", traces: "TraceInterner") -> np.ndarray:
    """SPAN (64 B) -> SPAN20 with the event interners (numpy reference of encode_spans20)."""
    out = np.zeros(spans.shape[0], dtype=SPAN20)
    out["ts_ns"] = spans["ts_ns"]
    out["trace_id"] = traces.ids(spans["trace_h"])
    cid = conns.ids(spans["conn_h"])
    sn = (spans["svc_id"].astype(np.uint32) << np.uint32(16)) | spans["node_id"].astype(np.uint32)
    out["ctx_id"] = ctxs.ids(spans["pod_id"], spans["pid"], cid, sn)
    out["group_id"] = spans["group_id"]
    return out


def compact_spans(spans: np.ndarray, interner: "ConnInterner") -> np.ndarray:
    """Spans keep the 64-byte layout; their conn key is rewritten to the same interned id."""
    out = spans.copy()
    out["conn_h"] = interner.ids(spans["conn_h"]).astype(np.uint64)
    return out


class CtxInterner:
    """(pod, pid, conn id, svc<<16|node) -> dense 24-bit context id; id 0 is the all-zero
    context. ``table()`` is the device context table (int32 [n, 4]) indexed by id. Ids are
    stable for the agent's lifetime, so the table only grows (and is re-uploaded then)."""

    MAX_IDS = 1 << 24

    def __init__(self):
        self._ids = {(0, 0, 0, 0): 0}
        self._rows = [(0, 0, 0, 0)]
        self._table = None

    def __len__(self) -> int:
        return len(self._rows)

    def ids(self, pod, pid, cid, sn) -> np.ndarray:
        rows = np.stack([np.asarray(x).astype(np.uint32) for x in (pod, pid, cid, sn)], axis=1)
        if rows.shape[0] == 0:
            return np.zeros(0, dtype=np.uint32)
        r64 = rows.astype(np.uint64)
        key = (r64[:, 0] * np.uint64(0x9E3779B97F4A7C15)) ^ (r64[:, 1] * np.uint64(0xC2B2AE3D27D4EB4F)) ^ \
              (r64[:, 2] * np.uint64(0x165667B19E3779F9)) ^ (r64[:, 3] * np.uint64(0xD6E8FEB86659FD93))
        _, first, inv = np.unique(key, return_index=True, return_inverse=True)
        uniq_rows = rows[first]
        if not np.array_equal(uniq_rows[inv], rows):  # 64-bit key collision: exact path
            uniq_rows, inv = np.unique(rows, axis=0, return_inverse=True)
        out = np.empty(uniq_rows.shape[0], dtype=np.uint32)
        for j, r in enumerate(map(tuple, uniq_rows.tolist())):
            v = self._ids.get(r)
            if v is None:
                v = len(self._rows)
                if v >= self.MAX_IDS:
                    raise OverflowError("more than 2^24 interned contexts")
                self._ids[r] = v
                self._rows.append(r)
                self._table = None
            out[j] = v
        return out[np.asarray(inv).reshape(-1)]

    def table(self) -> np.ndarray:
        if self._table is None:
            self._table = np.array(self._rows, dtype=np.uint32).reshape(-1, 4).view(np.int32)
        return self._table


class TraceInterner:
    """64-bit trace hash -> 32-bit id (0 = none), shared by a window's events and spans
    (numpy reference of the native encoder's trace table; no expiry)."""

    def __init__(self):
        self._ids = {}

    def ids(self, trace_h: np.ndarray) -> np.ndarray:
        uniq, inv = np.unique(np.asarray(trace_h, dtype=np.uint64), return_inverse=True)
        out = np.zeros(uniq.shape[0], dtype=np.uint32)
        for j, h in enumerate(uniq.tolist()):
            if h == 0:
                continue
            i = self._ids.get(h)
            if i is None:
                i = len(self._ids) + 1
                if i > TRACE_ID_MASK:  # 30-bit ids (EVENT16 keeps 2 bits for the epoch tag)
                    raise OverflowError("trace id space exhausted")
                self._ids[h] = i
            out[j] = i
        return out[np.asarray(inv).reshape(-1)]


def to_wire16(events: np.ndarray, conns: "ConnInterner", ctxs: "CtxInterner", traces: "TraceInterner"):
    """EVENT (64 B) -> (EVENT16 (16 B), t_base); spans must go through ``wire_spans`` with
    the same interners."""
    e20, t_base = to_wire20(events, conns, ctxs)
    out = np.zeros(events.shape[0], dtype=EVENT16)
    for f in ("ts_off", "ctx_type", "value_milli"):
        out[f] = e20[f]
    out["trace_id"] = traces.ids(events["trace_h"])
    return out, t_base


def wire_spans(spans: np.ndarray, conns: "ConnInterner", traces: "TraceInterner" = None) -> np.ndarray:
    """Spans for the compact wire formats: interned conn ids (and trace ids for EVENT16)."""
    out = compact_spans(spans, conns)
    if traces is not None:
        out["trace_h"] = traces.ids(spans["trace_h"]).astype(np.uint64)
    return out


def signal_scale_table() -> np.ndarray:
    """decode_scale per kernel signal type < 256 (1.0 for unknown types)."""
    scale = np.ones(256, dtype=np.float64)
    for s in catalog.SIGNALS:
        if s.kernel_type < 256:
            scale[s.kernel_type] = s.decode_scale
    return scale


def native_encoder():
    """The native WireEncoder (runtime/csrc/wire.h) configured with the signal catalogue."""
    from ..runtime import load

    return load().WireEncoder(milli_shift_table())


def string_hash64(s: str) -> int:
    """FNV-1a 64 of a string; 0 reserved for the empty string."""
    if not s:
        return 0
    h = 0xCBF29CE484222325
    for b in s.encode("utf-8"):
        h ^= b
        h = (h * 0x100000001B3) & ((1 << 64) - 1)
    return h or 1
