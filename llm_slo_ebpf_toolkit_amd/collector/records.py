"""Binary event/span record formats shared by the BPF probes, the native runtime and the GPU.

* ``REF_EVENT`` -- REF's packed 40-byte ``struct llm_slo_event``
  (ebpf/c/llm_slo_event.h:32-42). Accepted for replay compatibility; decoded with REF's
  exact rules (pkg/collector/ringbuf.go:152-243): type->(name, unit), count stays a count,
  cpu_steal stays raw ns, everything else ns/1e6 -> ms, conn tuple only if a port != 0
  (src_ip "0.0.0.0", protocol "tcp"), errno only if != 0, IPv4 little-endian bytes.
* ``EVENT`` -- 64-byte record: the probes' working record (probes/ebpf/mislo_record.h
  ``mislo_event``) and what user-space producers (the rocprofiler-sdk tool library,
  instrumented services, replay) push into the shared-memory rings. Every REF field plus
  interned workload ids (pod/node/service), a 64-bit trace-id hash, a 64-bit connection hash,
  a GPU id and flags.
* ``EVENT16`` -- the 16-byte record on the wire: the payload of every record the probes put on
  the BPF ring (``mislo_event16``), and what the agent's host encoder makes of user-space
  records. Timestamp as an epoch offset with a 2-bit epoch tag, workload identity as a context
  id into the device context table, fixed-point value, 30-bit trace id.
* ``DEF16`` -- the probes' id definition records on the same ring (same 16 bytes, type byte
  0xFE: a context row; 0xFD: a trace id), which the agent's consumer diverts to its tables.
* ``SPAN`` (64 B) / ``SPAN20`` -- spans as the span ring carries them / as the GPU join reads them.

``ProbeModel`` / ``HostEncoderModel`` are the numpy references of the in-kernel record path
(mislo_probe.h mislo_submit) and of the agent's host encoder (runtime/csrc/tables.h); the
native implementations are tested byte for byte against them.
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

TS_ZERO = 0xFFFFFFFF  # ts_off of a zero timestamp (never joins)

# 16-byte record (= probes/ebpf/mislo_record.h mislo_event16): ts = base[tag] + ts_off, the
# window carrying its last 4 epoch bases (counts[4..5], counts[8..13]); context id into the
# device context table; trace id shared with the window's spans (kernel ids < 2^24, ids the
# agent assigns >= 2^24).
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
DEF_TRACE, DEF_CTX, DEF_FIRST = 0xFD, 0xFE, 0xF0  # definition slot types (low byte of ctx_type)
DEF_PAD = 0xFC  # an unused slot of a batch flushed before it filled
KERNEL_CTX_LIMIT = 1 << 23     # kernel context ids 1 .. 2^23 - 1, host ids above
KERNEL_TRACE_LIMIT = 1 << 24   # kernel trace ids 1 .. 2^24 - 1, host ids above
CTX_IDS = 1 << 24
# 32-byte user-space record (probes/rocprof/mislo_rocprof.cpp, rings created with 32-byte
# records): what the GPU join needs of a user-space producer's event -- no connection, the
# value already in fixed point like the kernel's records, svc|node from the pod table. Half the
# PCIe bytes of EVENT; the agent takes either, per ring.
USER32 = np.dtype([
    ("ts_ns", "<i8"),        # 0  CLOCK_REALTIME ns
    ("trace_h", "<u8"),      # 8  trace hash (0 = none)
    ("value_milli", "<u4"),  # 16 value in 1/1000 of the signal's output unit (milli_int)
    ("pod_id", "<u4"),       # 20
    ("pid", "<u4"),          # 24
    ("signal_type", "u1"),   # 28
    ("flags", "u1"),         # 29 bit 0: has_gpu
    ("node_id", "<u2"),      # 30
])
assert USER32.itemsize == 32
# 24-byte user-space record (rings created with 24-byte records; ops/csrc/mislo_common.h
# User24): USER32 without the node id and flags the decode never reads, the timestamp as its
# low 44 bits (decoded to the value nearest the window's newest epoch base, +-2.4 h), pid < 2^22
# (Linux pid_max), pod id < 2^20 (the device pod table), signal type < 128. 25 % fewer PCIe
# bytes than USER32.
USER24 = np.dtype([
    ("trace_h", "<u8"),      # 0
    ("value_milli", "<u4"),  # 8
    ("ts_lo", "<u4"),        # 12 ts bits 0..31
    ("pid_sig", "<u4"),      # 16 pid | signal_type << 22 | ts_zero << 29 | has_gpu << 30
    ("pod_ts", "<u4"),       # 20 pod_id | (ts bits 32..43) << 20
])
assert USER24.itemsize == 24
USER24_TS_BITS = 44
# 16-byte user-space slot (rings created with 16-byte records; ops/csrc/mislo_common.h User16):
# USER24 without the trace hash. A record with a trace (pid_sig bit 31) is followed by a
# continuation slot {trace lo, trace hi, USER16_CONT, 0} that decodes as a hole; both are pushed
# in one batch, so a window never splits them. The GPU signals' records carry no trace unless the
# workload tagged its kernels (probes/rocprof mislo_rocprof_set_trace), so most take 16 bytes,
# two thirds of USER24. Signal type < 127 (127 with every other bit set would read as the marker).
USER16 = np.dtype([
    ("ts_lo", "<u4"),        # 0  ts bits 0..31
    ("value_milli", "<u4"),  # 4
    ("pid_sig", "<u4"),      # 8  pid | signal_type << 22 | ts_zero << 29 | has_gpu << 30 | has_trace << 31
    ("pod_ts", "<u4"),       # 12 pod_id | (ts bits 32..43) << 20
])
assert USER16.itemsize == 16
USER16_CONT = 0xFFFFFFFF
USER16_HAS_TRACE = 1 << 31

WIRE_DTYPES = {64: EVENT, 16: EVENT16}
RB_BUSY, RB_DISCARD, RB_HDR = 1 << 31, 1 << 30, 8   # BPF ring buffer record header bits
# A BPF ring record is a batch of BATCH_SLOTS 16-byte slots a CPU staged (probes/ebpf/mislo_probe.h
# mislo_stage_put): row r of a window is slot r % 8 of record r // 8
BATCH_SLOTS = 8
REC_PAYLOAD = 16 * BATCH_SLOTS                    # 128
REC_STRIDE = RB_HDR + REC_PAYLOAD                 # 136 ring bytes per record
PROBE_CPUS = 16                                   # the probe models' CPUs (a task runs on tid % 16)


def framed_rows(framed) -> int:
    """Rows (slots) of a framed image of whole batch records."""
    return len(framed) // REC_STRIDE * BATCH_SLOTS


def framed_slots(framed: np.ndarray):
    """(header len words per row [rows], slots as uint32 [rows, 4]) of a framed image."""
    r = np.ascontiguousarray(framed).view(np.uint32).reshape(-1, REC_STRIDE // 4)
    hdr = np.repeat(r[:, 0], BATCH_SLOTS)
    return hdr, r[:, 2:].reshape(-1, 4)


def framed_event_count(framed: np.ndarray) -> int:
    """Events in a framed image: event slots of committed (not busy / discarded) batch records."""
    hdr, sl = framed_slots(framed)
    return int(((hdr == REC_PAYLOAD) & ((sl[:, 1] & 0xFF) < DEF_FIRST)).sum())


def wire_bytes(wire: int) -> int:
    """PCIe bytes per event of wire code ``wire`` (64 = EVENT, 16 = EVENT16)."""
    if wire not in WIRE_DTYPES:
        raise ValueError(f"unknown wire code {wire}")
    return int(wire)


def wire_code(dtype: np.dtype) -> int:
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
    # 56 the request's retrieval time as the application reports it: REF's
    # llm.slo.retrieval.{vectordb,network,dns}_ms summed (demo/rag-service/main.go:393-397);
    # <= 0 / NaN = no breakdown (the application evidence of ops/csrc/posterior.hip)
    ("retr_ms", "<f4"),
    # 60 bit 0 (SPAN_LATE): the request's TTFT-SLO deadline (start + SLO) passed before the agent's
    # last window cut -- a breach that belongs to an earlier window (collector/otlp.py);
    # bit 1 (SPAN_NO_SLI): the request's SLI was counted by its first-token record already -- the
    # request span joins but does not count again; bit 2 (SPAN_FIRST_TOKEN): a first-token record
    # (exported when the first token is out, llm.slo.ttft_early) -- counted, and joined like the
    # request span (its keys but the connection: the request span brings the pod+conn tier), so the
    # request's kernel evidence reaches the window its SLI is counted in
    ("flags", "<u4"),
])
SPAN_LATE, SPAN_NO_SLI, SPAN_FIRST_TOKEN = 1, 2, 4
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


def to_user32(events: np.ndarray) -> np.ndarray:
    """64-byte EVENT records -> USER32 (mislo_rocprof.cpp emit with a 32-byte ring)."""
    out = np.zeros(len(events), dtype=USER32)
    st = events["signal_type"].astype(np.int64)
    out["ts_ns"] = events["ts_ns"]
    out["trace_h"] = events["trace_h"]
    out["value_milli"] = milli_int(events["value"], milli_shift_table()[np.clip(st, 0, 255)])
    out["pod_id"] = events["pod_id"]
    out["pid"] = events["pid"]
    out["signal_type"] = np.clip(st, 0, 255).astype(np.uint8)
    out["flags"] = ((events["flags"] >> 8) & 1).astype(np.uint8)
    out["node_id"] = events["node_id"]
    return out


def to_user24(events: np.ndarray) -> np.ndarray:
    """64-byte EVENT records -> USER24 (mislo_rocprof.cpp emit with a 24-byte ring). Raises on
    a pid, pod id or signal type that does not fit the record."""
    st = events["signal_type"].astype(np.int64)
    pid = events["pid"].astype(np.uint64)
    pod = events["pod_id"].astype(np.uint64)
    if len(events) and (pid.max() >= 1 << 22 or pod.max() >= 1 << 20 or st.max() >= 128 or st.min() < 0):
        raise ValueError("USER24 holds pid < 2^22, pod id < 2^20, signal type < 128")
    ts = events["ts_ns"].astype(np.int64)
    t = ts.astype(np.uint64)
    out = np.zeros(len(events), dtype=USER24)
    out["trace_h"] = events["trace_h"]
    out["value_milli"] = milli_int(events["value"], milli_shift_table()[np.clip(st, 0, 255)])
    out["ts_lo"] = (t & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    zero = (ts == 0).astype(np.uint64)
    gpu = ((events["flags"].astype(np.uint64) >> np.uint64(8)) & np.uint64(1))
    out["pid_sig"] = (pid | (st.astype(np.uint64) << np.uint64(22)) | (zero << np.uint64(29))
                      | (gpu << np.uint64(30))).astype(np.uint32)
    out["pod_ts"] = (pod | (((t >> np.uint64(32)) & np.uint64(0xFFF)) << np.uint64(20))).astype(np.uint32)
    return out


def to_user16(events: np.ndarray) -> np.ndarray:
    """64-byte EVENT records -> USER16 slots (a traced record takes two: the record, then its
    trace in a continuation slot). Raises like ``to_user24`` and on signal type 127."""
    u24 = to_user24(events)
    st = events["signal_type"].astype(np.int64)
    if len(events) and st.max() >= 127:
        raise ValueError("USER16 holds signal type < 127")
    traced = u24["trace_h"] != 0
    n = len(u24) + int(traced.sum())
    out = np.zeros(n, dtype=USER16)
    pos = np.arange(len(u24)) + np.concatenate([[0], np.cumsum(traced)[:-1]]).astype(np.int64) if len(u24) else \
        np.zeros(0, np.int64)
    out["ts_lo"][pos] = u24["ts_lo"]
    out["value_milli"][pos] = u24["value_milli"]
    out["pid_sig"][pos] = u24["pid_sig"] | np.where(traced, np.uint32(USER16_HAS_TRACE), np.uint32(0))
    out["pod_ts"][pos] = u24["pod_ts"]
    cont = pos[traced] + 1
    th = u24["trace_h"][traced].astype(np.uint64)
    out["ts_lo"][cont] = (th & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    out["value_milli"][cont] = (th >> np.uint64(32)).astype(np.uint32)
    out["pid_sig"][cont] = np.uint32(USER16_CONT)
    return out


def user16_to_user24(u: np.ndarray):
    """USER16 slots -> (USER24 rows, one per slot, and the continuation mask: those rows are
    holes). A record's trace comes from the slot after it."""
    cont = u["pid_sig"] == np.uint32(USER16_CONT)
    v = np.zeros(len(u), dtype=USER24)
    v["ts_lo"], v["value_milli"], v["pod_ts"] = u["ts_lo"], u["value_milli"], u["pod_ts"]
    v["pid_sig"] = u["pid_sig"] & np.uint32(0x7FFFFFFF)
    has = ((u["pid_sig"] & np.uint32(USER16_HAS_TRACE)) != 0) & ~cont
    nxt = np.minimum(np.arange(len(u)) + 1, max(len(u) - 1, 0))
    ok = has & (np.arange(len(u)) + 1 < len(u))
    ok &= cont[nxt] if len(u) else ok
    tr = (u["value_milli"][nxt].astype(np.uint64) << np.uint64(32)) | u["ts_lo"][nxt].astype(np.uint64)
    v["trace_h"] = np.where(ok, tr, np.uint64(0))
    return v, cont


def user24_ts(u: np.ndarray, base: int) -> np.ndarray:
    """USER24 timestamps: the value nearest ``base`` with the record's low 44 bits (0 when the
    record says it has none); ops/csrc/mislo_common.h user24_ts."""
    t44 = ((u["pod_ts"].astype(np.uint64) >> np.uint64(20)) << np.uint64(32)) | u["ts_lo"].astype(np.uint64)
    mask = np.uint64((1 << USER24_TS_BITS) - 1)
    d = (t44 - np.uint64(base & 0xFFFFFFFFFFFFFFFF)) & mask
    sh = np.uint64(64 - USER24_TS_BITS)
    sd = ((d << sh).view(np.int64) >> np.int64(64 - USER24_TS_BITS))
    ts = np.int64(base) + sd
    return np.where((u["pid_sig"] >> np.uint32(29)) & np.uint32(1), np.int64(0), ts).astype(np.int64)


def user24_to_user32(u: np.ndarray, base: int) -> np.ndarray:
    """USER24 -> USER32 (timestamps nearest ``base``; node id 0: USER24 does not carry it)."""
    pid_sig, pod_ts = u["pid_sig"].astype(np.uint32), u["pod_ts"].astype(np.uint32)
    v = np.zeros(len(u), dtype=USER32)
    v["ts_ns"] = user24_ts(u, int(base))
    v["trace_h"] = u["trace_h"]
    v["value_milli"] = u["value_milli"]
    v["pod_id"] = pod_ts & np.uint32(0xFFFFF)
    v["pid"] = pid_sig & np.uint32(0x3FFFFF)
    v["signal_type"] = ((pid_sig >> np.uint32(22)) & np.uint32(0x7F)).astype(np.uint8)
    v["flags"] = ((pid_sig >> np.uint32(30)) & np.uint32(1)).astype(np.uint8)
    return v


def to_user(events: np.ndarray, rec: int) -> np.ndarray:
    """EVENT records -> what a user-space producer writes into a ``rec``-byte ring."""
    if rec == 64:
        return events
    if rec == 32:
        return to_user32(events)
    if rec == 24:
        return to_user24(events)
    if rec == 16:
        return to_user16(events)
    raise ValueError(f"user-space records are 64, 32, 24 or 16 bytes, not {rec}")


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




def conn32_np(keys: np.ndarray) -> np.ndarray:
    """The 32-bit connection identity of context rows (runtime/csrc/records.h conn32, the
    kernel's mislo_conn32): fold of the 64-bit connection key, forced odd; 0 = no connection."""
    k = np.asarray(keys, dtype=np.uint64)
    f = ((k ^ (k >> np.uint64(32))) & np.uint64(0xFFFFFFFF)) | np.uint64(1)
    return np.where(k == 0, np.uint64(0), f).astype(np.uint32)


def conn32(key: int) -> int:
    key = int(key)
    return 0 if key == 0 else (((key ^ (key >> 32)) & 0xFFFFFFFF) | 1)


# 20-byte span record (ops/csrc SpanC20, runtime/csrc/records.h Span20): what the GPU join reads of
# a span, with (pod, pid, conn32, svc|node) as a context id and a trace id from the events' id space.
SPAN20 = np.dtype({"names": ["ts_ns", "trace_id", "ctx_id", "group_id"],
                   "formats": ["<i8", "<u4", "<u4", "<u4"], "offsets": [0, 8, 12, 16], "itemsize": 20})


def epoch_offset(ts: int, base: int) -> int:
    """mislo_submit / EpochClock.stamp: offset of ts from an epoch base (clamped)."""
    if ts == 0:
        return TS_ZERO
    if ts < base:
        return 0
    return min(ts - base, TS_ZERO - 1)


class ProbeModel:
    """numpy/Python reference of the probes' in-kernel record path (probes/ebpf/mislo_probe.h
    mislo_emit -> mislo_submit; runtime/csrc/probesim.h is the native model tested against it):
    floors, context and trace interning with the definition record emitted ahead of the first
    use, epoch-relative timestamps with the published epoch's tag. ``cfg`` is the mislo_cfg
    array (uint64[128])."""

    CFG_EPOCH, CFG_TRACE_NEXT, CFG_CTX_NEXT = 124, 125, 126

    def __init__(self, cfg: np.ndarray = None, cpus: int = PROBE_CPUS):
        self.cfg = cfg if cfg is not None else np.zeros(128, dtype=np.uint64)
        self.ctx = {}
        self.traces = {}
        self.stages = [([], 0) for _ in range(max(1, cpus))]  # per CPU: (slots, epoch)

    def _flush(self, cpu: int, out: list) -> None:
        sl, _ = self.stages[cpu]
        if sl:
            out.extend(sl + [(0, DEF_PAD, 0, 0)] * (BATCH_SLOTS - len(sl)))
        self.stages[cpu] = ([], 0)

    def _put(self, cpu: int, slot: tuple, flush_now: bool, out: list) -> None:
        """mislo_stage_put: into the CPU's batch; the batch goes out when full, with a definition,
        or before a slot of a newer epoch."""
        epoch = int(self.cfg[self.CFG_EPOCH])
        sl, ep = self.stages[cpu]
        if sl and ep != epoch:
            self._flush(cpu, out)
        sl = self.stages[cpu][0] + [slot]
        self.stages[cpu] = (sl, epoch)
        if len(sl) == BATCH_SLOTS or flush_now:
            self._flush(cpu, out)

    def flush(self) -> np.ndarray:
        """The agent's cut: every CPU's partial batch, CPU 0 first."""
        out = []
        for c in range(len(self.stages)):
            self._flush(c, out)
        return self._as_slots(out)

    @staticmethod
    def _as_slots(out):
        return np.array(out, dtype=np.uint32).reshape(-1, 4).view(EVENT16).reshape(-1) if out else \
            np.zeros(0, dtype=EVENT16)

    def encode(self, events: np.ndarray, flush: bool = True) -> np.ndarray:
        """Ring payloads (whole batches of EVENT16 slots, definitions and pads included, ring
        order) for ``events``; with ``flush`` the partial batches too."""
        out = []
        shift = milli_shift_table()
        for e in events:
            cpu = int(e["tid"]) % len(self.stages)
            st = int(e["signal_type"])
            if st < 120 and int(e["value"]) < int(self.cfg[2 + st]):
                continue
            ck = int(e["conn_h"]) or conn_hash(int(e["src_port"]), int(e["dst_port"]), int(e["dst_ip"]))
            c = conn32(ck)
            pod, pid = int(e["pod_id"]), int(e["pid"])
            ctx = 0
            if pod or pid or c:
                ctx = self.ctx.get((pod, pid, c), 0)
                if not ctx:
                    fresh = int(self.cfg[self.CFG_CTX_NEXT]) + 1
                    self.cfg[self.CFG_CTX_NEXT] = fresh
                    if fresh < KERNEL_CTX_LIMIT:
                        self._put(cpu, (c, DEF_CTX | (fresh << 8), pod, pid), True, out)
                        self.ctx[(pod, pid, c)] = fresh
                        ctx = fresh
            tid = 0
            th = int(e["trace_h"])
            if th:
                tid = self.traces.get(th, 0)
                if not tid:
                    fresh = int(self.cfg[self.CFG_TRACE_NEXT])
                    self.cfg[self.CFG_TRACE_NEXT] = fresh + 1
                    tid = fresh % (KERNEL_TRACE_LIMIT - 1) + 1
                    self._put(cpu, (tid, DEF_TRACE, th & 0xFFFFFFFF, th >> 32), True, out)
                    self.traces[th] = tid
            epoch = int(self.cfg[self.CFG_EPOCH])
            milli = int(milli_int(np.array([int(e["value"])], dtype=np.uint64),
                                  np.array([shift[st] if st < 256 else 3], dtype=np.int8))[0])
            self._put(cpu, (epoch_offset(int(e["ts_ns"]), epoch & ~3), (st & 0xFF) | (ctx << 8), milli,
                            (tid & TRACE_ID_MASK) | ((epoch & 3) << EPOCH_TAG_SHIFT)), False, out)
        if flush:
            for c in range(len(self.stages)):
                self._flush(c, out)
        return self._as_slots(out)


def frame(payloads: np.ndarray) -> np.ndarray:
    """Committed BPF ring records (8-byte header {len = 128, pg_off = 0} + a batch of 8 EVENT16
    slots) for whole batches of slots."""
    p = np.ascontiguousarray(payloads).view(np.uint32).reshape(-1, 4)
    if p.shape[0] % BATCH_SLOTS:
        raise ValueError("frame: whole batches of 8 slots only")
    out = np.zeros((p.shape[0] // BATCH_SLOTS, REC_STRIDE // 4), dtype=np.uint32)
    out[:, 0] = REC_PAYLOAD
    out[:, 2:] = p.reshape(-1, REC_PAYLOAD // 4)
    return out.view(np.uint8).reshape(-1)


def unframe(image: np.ndarray):
    """libbpf ring_buffer__consume semantics over a byte image of consecutive records starting at a
    record boundary: (EVENT16 event slots, definition slots, n_discarded, stopped_at_busy); pads
    are dropped."""
    b = np.ascontiguousarray(image).view(np.uint8)
    off, ev, defs, disc = 0, [], [], 0
    while off + RB_HDR <= b.size:
        ln = int(b[off:off + 4].view(np.uint32)[0])
        if ln & RB_BUSY:
            return _as16(ev), _as16(defs), disc, True
        plen = ln & ~(RB_BUSY | RB_DISCARD)
        if ln & RB_DISCARD:
            disc += 1
        elif plen == REC_PAYLOAD:
            for j in range(BATCH_SLOTS):
                rec = tuple(int(x) for x in b[off + 8 + 16 * j:off + 24 + 16 * j].view(np.uint32))
                t = rec[1] & 0xFF
                if t != DEF_PAD:
                    (defs if t >= DEF_FIRST else ev).append(rec)
        off += (plen + RB_HDR + 7) & ~7
    return _as16(ev), _as16(defs), disc, False


def _as16(rows):
    return np.array(rows, dtype=np.uint32).reshape(-1, 4).view(EVENT16).reshape(-1) if rows else \
        np.zeros(0, dtype=EVENT16)


class HostEncoderModel:
    """Python reference of the agent's id tables and host encoder (runtime/csrc/tables.h
    AgentTables): kernel context rows from definitions (svc|node from pod metadata), host context
    ids from 2^23, trace ids shared with the kernel's definitions (host ids from 2^24), EVENT16
    with per-record epoch choice, SPAN20, and the row patch in queue order."""

    def __init__(self):
        self.pod_sn = {}
        self.kernel_rows = {}
        self.host = {}
        self.host_next = KERNEL_CTX_LIMIT
        self.traces = {}
        self.trace_next = KERNEL_TRACE_LIMIT
        self.pending = []

    def set_pod(self, pod: int, sn: int) -> None:
        if self.pod_sn.get(pod, 0) == sn:
            return
        self.pod_sn[pod] = sn
        for cid in sorted(self.kernel_rows):
            r = self.kernel_rows[cid]
            if r[0] == pod and (r[0] | r[1] | r[2]):
                r = (r[0], r[1], r[2], sn)
                self.kernel_rows[cid] = r
                self.pending.append((cid, r))

    def apply_defs(self, defs: np.ndarray) -> None:
        for d in np.ascontiguousarray(defs).view(np.uint32).reshape(-1, 4).tolist():
            t = d[1] & 0xFF
            if t == DEF_CTX:
                cid = d[1] >> 8
                if 0 < cid < KERNEL_CTX_LIMIT:
                    r = (d[2], d[3], d[0], self.pod_sn.get(d[2], 0))
                    self.kernel_rows[cid] = r
                    self.pending.append((cid, r))
            elif t == DEF_TRACE and 0 < d[0] < KERNEL_TRACE_LIMIT:
                self.traces[d[2] | (d[3] << 32)] = d[0]

    def trace_id(self, h: int) -> int:
        h = int(h)
        if not h:
            return 0
        if h not in self.traces:
            self.traces[h] = self.trace_next
            self.trace_next = KERNEL_TRACE_LIMIT if self.trace_next == TRACE_ID_MASK else self.trace_next + 1
        return self.traces[h]

    def host_ctx(self, pod, pid, c, sn) -> int:
        key = (int(pod), int(pid), int(c), int(sn))
        if key == (0, 0, 0, 0):
            return 0
        if key not in self.host:
            self.host[key] = self.host_next
            self.pending.append((self.host_next, key))
            self.host_next += 1
        return self.host[key]

    def encode_events(self, events: np.ndarray, bases) -> np.ndarray:
        b = (list(bases) + [0, 0, 0, 0])[:4]
        shift = milli_shift_table()
        live = [j for j in range(4) if b[j] != 0]
        oldest = min(live, key=lambda j: (b[j], j)) if live else 0
        out = np.zeros(events.shape[0], dtype=EVENT16)
        for i, e in enumerate(events):
            ts = int(e["ts_ns"])
            cands = [j for j in live if ts >= b[j]]
            tag = max(cands, key=lambda j: (b[j], j)) if cands else oldest
            st = int(e["signal_type"])
            ck = int(e["conn_h"]) or conn_hash(int(e["src_port"]), int(e["dst_port"]), int(e["dst_ip"]))
            sn = (int(e["svc_id"]) << 16) | int(e["node_id"])
            ctx = self.host_ctx(e["pod_id"], e["pid"], conn32(ck), sn)
            milli = int(milli_int(np.array([int(e["value"])], dtype=np.uint64),
                                  np.array([shift[st] if st < 256 else 3], dtype=np.int8))[0])
            out[i] = (epoch_offset(ts, b[tag]), (st & 0xFF) | (ctx << 8), milli,
                      (self.trace_id(e["trace_h"]) & TRACE_ID_MASK) | (tag << EPOCH_TAG_SHIFT))
        return out

    def encode_spans(self, spans: np.ndarray) -> np.ndarray:
        out = np.zeros(spans.shape[0], dtype=SPAN20)
        for i, s in enumerate(spans):
            sn = (int(s["svc_id"]) << 16) | int(s["node_id"])
            out[i] = (int(s["ts_ns"]), self.trace_id(s["trace_h"]),
                      self.host_ctx(s["pod_id"], s["pid"], conn32(int(s["conn_h"])), sn), int(s["group_id"]))
        return out

    def take_rows(self):
        ids = np.array([p[0] for p in self.pending], dtype=np.uint32)
        rows = np.array([p[1] for p in self.pending], dtype=np.uint32).reshape(-1, 4)
        self.pending = []
        return ids, rows


def native_tables():
    """The agent's native id tables / host encoder (runtime/csrc/tables.h)."""
    from ..runtime import load

    return load().AgentTables(milli_shift_table())


def string_hash64(s: str) -> int:
    """FNV-1a 64 of a string; 0 reserved for the empty string."""
    if not s:
        return 0
    h = 0xCBF29CE484222325
    for b in s.encode("utf-8"):
        h ^= b
        h = (h * 0x100000001B3) & ((1 << 64) - 1)
    return h or 1
