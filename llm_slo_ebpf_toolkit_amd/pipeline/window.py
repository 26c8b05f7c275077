"""Per-GPU window pipeline: copy stream || compute stream || RCCL side stream.

One process drives one MI355X. For window i (nb-buffered device I/O, b = i % nb, nb = 3):

    copy stream    : H2D records(i) -> ev[b]; [counts|labels|spans](i) -> aux[b] (PCIe DMA)
    compute stream : wait H2D(i); decode -> partition -> LDS join -> finalize ->
                     MFMA posterior + confusion -> MFMA sufficient stats -> pack(packet[b])
    comm stream    : wait compute(i); all_reduce(packet[b]) over RCCL/xGMI;
                     totals += packet[b]; packet_host[b] <- packet[b] (async D2H)

so the H2D of window i+1 and the node-wide all-reduce of window i run underneath the
kernels of window i+1. The host then folds window i-1's all-reduced statistics into the
online model (learned Bayes from random-init priors, or LDA) and uploads it with a
stream-ordered copy, so window i+1 is scored by a model fitted on windows <= i-1
(prequential, never on its own labels). Every rank refits from the same all-reduced
totals, so the model stays identical across the node without a broadcast.

The packet (see ops/csrc/bindings.cpp) packs signal histograms, status counters, debug
pair counters, the confusion matrix and the 32x32 f64 sufficient statistics into one
12.9 KB buffer: a single latency-bound collective per window instead of five.
"""

from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from ..collector import records
from ..models.bayes import LDA, N_DOMAINS, NaiveBayes, SufficientStats
from ..models.metrics import macro_f1_from_confusion
from ..ops.engine import GpuEngine, decode_debug, model_bytes
from ..signals import catalog

_HOST_TRACE = bool(__import__("os").environ.get("MISLO_HOST_TRACE"))

PACKET_LAYOUT = (256, 48, 18, 8, 256, 1024, 16)  # hist, status, misc(+16 value sums), dbg, confusion, stats, count


def unpack_packet(p: np.ndarray) -> Dict[str, np.ndarray]:
    o = 0
    out = {}
    for name, n in zip(("hist", "status", "misc", "dbg", "confusion", "stats", "count"), PACKET_LAYOUT):
        out[name] = p[o:o + n]
        o += n
    out["hist"] = out["hist"].reshape(16, 16)
    out["status"] = out["status"].reshape(16, 3)
    out["confusion"] = out["confusion"].reshape(16, 16)
    out["stats"] = out["stats"].reshape(32, 32)
    out["value_sum"] = out["misc"][2:18] * 1e-3  # per-slot sums of decoded values (output units)
    return out


def stats_from_packet(p: Dict[str, np.ndarray]) -> SufficientStats:
    st = p["stats"]
    D = N_DOMAINS
    return SufficientStats(count=p["count"][:D].copy(), elevated_sum=st[:16, :D].copy(),
                           x_sum=st[16:, :D].copy(), xx=st[16:, 16:].copy())


def aux_head(group_cap: int) -> int:
    """Bytes ahead of the spans in a packed input block: counts int32[16], labels int32[G],
    padded to 64 so the span records stay 64-byte aligned."""
    return (4 * records.COUNTS_LEN + 4 * max(int(group_cap), 1) + 63) // 64 * 64


@dataclass
class StagedWindow:
    """A window's records in pinned host memory, ready for DMA."""
    ev: "object"        # torch uint8 pinned [>= n_events*wire]
    sp: "object"        # torch uint8 pinned [>= n_spans*64]
    counts: "object"    # torch int32 pinned [8]: n_ev, n_spans, n_groups, n_local, t_base lo/hi, n_ctx
    labels: "object"    # torch int32 pinned [group_cap]
    n_events: int
    n_spans: int
    n_groups: int
    group_domains: List[List[str]] = field(default_factory=list)
    wire: int = 64                      # event record bytes: 64 (EVENT), 32 (EVENT32), 20 (EVENT20)
    pod_table: Optional[np.ndarray] = None  # int32 pod id -> svc<<16|node (wire 32)
    ctx_rows: "object" = None           # torch int32 pinned [n_ctx, 4] context table snapshot (wire 20/16)
    n_ctx: int = 0
    encode_s: float = 0.0               # host time spent converting records to the wire format
    # pinned [counts | labels | pad | spans] block when counts / labels / sp are views of it
    # (WireStager): the three small inputs then cross PCIe as ONE copy (aux_head(group_cap))
    aux: "object" = None
    span_bytes: int = 64                # 20 = SPAN20 records (counts[7]), else 64-byte SPAN


def stage_window(torch, events: np.ndarray, spans: np.ndarray, n_groups: int, labels: Optional[np.ndarray],
                 group_cap: int, group_domains=None, wire: int = 64, interner=None,
                 n_local: Optional[int] = None, ctx_interner=None, trace_interner=None,
                 encoder=None) -> StagedWindow:
    """Pin a window for DMA. ``wire=32`` converts 64-byte events to the compact 32-byte
    record (interned conn ids, milli-unit values; collector/records.py EVENT32), halving
    the PCIe bytes that bound the pipeline. ``wire=20`` / ``16`` go further (EVENT20 /
    EVENT16: window-relative timestamps, interned (pod, pid, conn, svc|node) contexts whose
    rows travel once, appended to a device table; EVENT16 also interns trace hashes). Spans
    get the same interned ids. 20/16 use the native ``encoder`` (records.native_encoder(),
    one per record stream, written straight into pinned memory) unless numpy interners are
    given (the reference path the tests compare against)."""
    t_enc = time.perf_counter()
    pod_tab = None
    ctx_rows, n_ctx, t_base = None, 0, 0
    if wire in (20, 16, records.WIRE_20T) and ctx_interner is None and events.dtype == records.EVENT:
        enc = encoder if encoder is not None else records.native_encoder()
        ev = torch.empty(max(events.shape[0], 1) * records.wire_bytes(wire), dtype=torch.uint8).pin_memory()
        sp = torch.empty(max(spans.shape[0], 1) * 64, dtype=torch.uint8).pin_memory()
        t_enc = time.perf_counter()  # conversion only (the agent reuses its pinned buffers)
        try:
            t_base = enc.encode(np.ascontiguousarray(events), ev.numpy(), wire)
        except ValueError:
            # the window's timestamps span >= 2^32 ns (late / skewed producers): this window
            # travels as 32-byte records, which carry absolute timestamps
            wire = 32
        else:
            enc.encode_spans(np.ascontiguousarray(spans), sp.numpy(), wire in (16, records.WIRE_20T))
            if wire != records.WIRE_20T:  # kernel-interned trace ids live as long as the LRU keeps them
                enc.end_window()
            tab = enc.ctx_table()
            n_ctx = int(tab.shape[0])
            ctx_rows = torch.from_numpy(tab).pin_memory()
            return _finish_stage(torch, ev, sp, events.shape[0], spans.shape[0], n_groups, labels, group_cap,
                                 group_domains, wire, None, ctx_rows, n_ctx, t_base, n_local, t_enc)
    if wire in (32, 20, 16, records.WIRE_20T):
        if interner is None:
            interner = records.ConnInterner()
        if wire == 32 and events.dtype == records.EVENT:
            pod_tab = records.pod_table(events, spans)
            events = records.to_compact(events, interner)
        elif wire in (20, 16, records.WIRE_20T):
            if wire == 20:
                events, t_base = records.to_wire20(events, interner, ctx_interner)
            elif wire == records.WIRE_20T:
                trace_interner = trace_interner if trace_interner is not None else records.TraceInterner()
                events = records.to_wire20t(events, interner, ctx_interner, trace_interner)
            else:
                trace_interner = trace_interner if trace_interner is not None else records.TraceInterner()
                events, t_base = records.to_wire16(events, interner, ctx_interner, trace_interner)
            tab = ctx_interner.table()
            n_ctx = int(tab.shape[0])
            ctx_rows = torch.from_numpy(tab.copy()).pin_memory()
        spans = records.wire_spans(spans, interner, trace_interner if wire in (16, records.WIRE_20T) else None)
    elif wire != 64:
        raise ValueError("wire must be 64, 32, 21 (EVENT20T), 20 or 16")
    ev = torch.from_numpy(events.view(np.uint8).reshape(-1).copy()).pin_memory()
    sp = torch.from_numpy(spans.view(np.uint8).reshape(-1).copy()).pin_memory()
    return _finish_stage(torch, ev, sp, events.shape[0], spans.shape[0], n_groups, labels, group_cap,
                         group_domains, wire, pod_tab, ctx_rows, n_ctx, t_base, n_local, t_enc)


def _finish_stage(torch, ev, sp, n_ev: int, n_sp: int, n_groups: int, labels, group_cap: int, group_domains,
                  wire: int, pod_tab, ctx_rows, n_ctx: int, t_base: int, n_local, t_enc: float) -> StagedWindow:
    # counts[3] = node-local events; events[n_local:] are imported halo / remote-trace
    # records that join but are not counted (decode kernels, parallel/exchange.py)
    nl = 0 if n_local is None or n_local >= n_ev else int(n_local)
    counts = torch.from_numpy(records.counts_row(n_ev, n_sp, n_groups, nl, (t_base,), n_ctx).copy()).pin_memory()
    lab = np.full(group_cap, -1, dtype=np.int32)
    if labels is not None:
        lab[: len(labels)] = labels
    labels_t = torch.from_numpy(lab).pin_memory()
    return StagedWindow(ev, sp, counts, labels_t, int(n_ev), int(n_sp), n_groups, list(group_domains or []), wire,
                        pod_tab, ctx_rows, n_ctx, time.perf_counter() - t_enc)


class WireStager:
    """The agent's per-window host stage: 64-byte probe records (as the probes write them into
    the ring) -> 16/20-byte wire records in one of two reusable pinned slots, on the native
    encoder's worker pool (runtime/csrc/wire.h ``encode_window``). Window k writes slot k % nb,
    the buffer the pipeline's H2D of window k reads, after the H2D of window k - nb (the slot's
    previous reader) has completed, so encoding window k+1 overlaps the GPU work of window k.

    ``wire=64`` ships the ring records unchanged: ``events``/``spans`` must then already sit in
    pinned memory (the probe ring is pinned), and staging only fills the counts and labels.

    ``wire=32`` / ``24`` are the probes' own compact records (probes/ebpf/mislo_record.h
    ``mislo_event32``: the kernel interns connections and converts values to fixed point;
    ``mislo_event24``: it also interns the (pod, pid, conn, svc|node) context), so events also
    DMA straight from the pinned ring. The host maps the window's spans onto the same
    connection ids (``self.enc`` mirrors the kernel's maps; ``probe_records`` writes a replayed
    ring with it) and ships the pod table (32) or the new context rows (24) when they change."""

    def __init__(self, torch, pipe: "WindowPipeline", sig_cap: int, span_cap: int, group_cap: int, wire: int = 16,
                 threads: int = 8):
        if wire not in (16, 20, records.WIRE_20T, 24, 32, 64):
            raise ValueError("WireStager: wire must be 16, 20, 21 (EVENT20T), 24, 32 or 64")
        self.torch, self.pipe, self.wire, self.threads = torch, pipe, wire, max(1, int(threads))
        self.group_cap = group_cap
        pin = lambda n, dt=torch.uint8: torch.empty(n, dtype=dt).pin_memory()  # noqa: E731
        self.enc = records.native_encoder() if wire != 64 else None
        self.nb = pipe.nb  # one pinned slot per device buffer of the pipeline
        self.ev = [pin(max(sig_cap, 1) * wire) for _ in range(self.nb)] if wire in (16, 20) else None
        # [counts | labels | pad | spans] per slot: one H2D for the window's small inputs
        head = aux_head(group_cap)
        self.aux = [pin(head + max(span_cap, 1) * 64) for _ in range(self.nb)] if wire != 64 else None
        self.sp = [a[head:] for a in self.aux] if wire != 64 else None
        if self.aux is not None:
            cb = 4 * records.COUNTS_LEN
            self.counts = [a[:cb].view(torch.int32) for a in self.aux]
            self.labels = [a[cb:cb + 4 * max(group_cap, 1)].view(torch.int32) for a in self.aux]
        else:
            self.counts = [pin(records.COUNTS_LEN, torch.int32) for _ in range(self.nb)]
            self.labels = [pin(group_cap, torch.int32) for _ in range(self.nb)]
        self.ctx = pin((1 << 16) * 4, torch.int32).view(-1, 4) if wire in (16, 20, records.WIRE_20T, 24) else None
        self.n_ctx = 1
        self.k = 0
        self.encode_s = 0.0

    def probe_records(self, events: np.ndarray):
        """EVENT32 / EVENT24 records (``self.wire``) for 64-byte ``events`` as the probes emit
        them (kernel-side connection / context interning, integer fixed point), written into
        pinned memory: a replayed ring."""
        if self.wire not in (records.WIRE_20T, 24, 32):
            raise ValueError("probe_records: wire 21 (EVENT20T), 24 or 32")
        out = self.torch.empty(max(events.shape[0], 1) * records.wire_bytes(self.wire),
                               dtype=self.torch.uint8).pin_memory()
        self.enc.encode(np.ascontiguousarray(events), out.numpy(), self.wire)
        return out

    def probe_ring16(self, events: np.ndarray, epoch_ns: int = 0):
        """EVENT16 records for 64-byte ``events`` as the probes write them with
        -DMISLO_RING_EVENT16 (kernel-interned contexts and trace ids, offsets from the epoch the
        agent last published, tagged with it), in pinned memory, plus the window's epoch bases.
        ``epoch_ns`` > 0 publishes a new epoch every ``epoch_ns`` inside the window (tags 0-3)."""
        if self.wire != 16:
            raise ValueError("probe_ring16: wire 16")
        ev = np.zeros(events.shape[0], dtype=records.EVENT16)
        t_base = int(self.enc.encode(np.ascontiguousarray(events), ev.view(np.uint8).reshape(-1), 16))
        bases = (t_base,)
        if epoch_ns > 0:
            ev, bases = records.retag_epochs(ev, t_base, epoch_ns)
        out = self.torch.from_numpy(ev.view(np.uint8).reshape(-1).copy()).pin_memory()
        return out, bases

    def stage(self, events: np.ndarray, spans: np.ndarray, n_groups: int, labels: Optional[np.ndarray],
              group_domains=None, n_local: Optional[int] = None, ev_pinned=None, sp_pinned=None,
              pod_table: Optional[np.ndarray] = None, bases=None) -> StagedWindow:
        """One window into slot k % nb. ``ev_pinned``: the pinned probe ring segment for wire
        64/32/24/21, and for wire 16 when the probes write EVENT16 (then ``bases`` = the window's
        epoch bases); without it wire 16/20 encode the 64-byte records here."""
        torch = self.torch
        slot = self.k % self.nb
        if self.k >= self.nb:  # slot's previous reader: the H2D of window k - nb
            self.pipe.h2d_done[slot].synchronize()
        t0 = time.perf_counter()
        n_ev, n_sp = int(events.shape[0]), int(spans.shape[0])
        t_base = 0
        span_bytes = 64
        if self.wire == 16 and ev_pinned is not None:  # probe-native EVENT16 ring
            ev, sp = ev_pinned, self.sp[slot]
            if n_sp * 20 > sp.numel():
                raise ValueError("window exceeds the stager's capacity")
            # spans as 20-byte SPAN20 on the kernel's trace ids and context ids
            self.enc.encode_spans20(spans, sp.numpy()[: n_sp * 20])
            span_bytes = 20
            bases = tuple(bases) if bases is not None else (0,)
        elif self.wire == 64:
            ev, sp = ev_pinned, sp_pinned
            if ev is None or sp is None:
                raise ValueError("wire 64 stages the pinned ring records: pass ev_pinned / sp_pinned")
        elif self.wire in (records.WIRE_20T, 24, 32):
            ev, sp = ev_pinned, self.sp[slot]
            if ev is None or (self.wire == 32 and pod_table is None):
                raise ValueError("wire 32/24/21 stage the pinned probe ring: pass ev_pinned (and pod_table for 32)")
            if n_sp * 64 > sp.numel():
                raise ValueError("window exceeds the stager's capacity")
            # spans onto the kernel's connection ids (EVENT20T: 20-byte SPAN20 on its trace and
            # context ids)
            if self.wire == records.WIRE_20T:
                self.enc.encode_spans20(spans, sp.numpy()[: n_sp * 20])
                span_bytes = 20
            else:
                self.enc.encode_spans(spans, sp.numpy(), False)
        else:
            ev, sp = self.ev[slot], self.sp[slot]
            if n_ev * self.wire > ev.numel() or n_sp * 64 > sp.numel():
                raise ValueError("window exceeds the stager's capacity")
            t_base = self.enc.encode_window(events, ev.numpy(), self.wire, spans, sp.numpy(), self.threads)
            self.enc.end_window()
        if self.ctx is not None:
            n_ctx = int(self.enc.n_ctx)
            if n_ctx > self.n_ctx:  # new context rows (append-only: rows < n_ctx never change)
                if n_ctx > self.ctx.shape[0]:
                    cap = 1 << int(np.ceil(np.log2(n_ctx)))
                    grown = torch.empty(cap * 4, dtype=torch.int32).pin_memory().view(-1, 4)
                    grown[: self.n_ctx].copy_(self.ctx[: self.n_ctx])
                    self.ctx = grown
                self.ctx.numpy()[self.n_ctx:n_ctx] = self.enc.ctx_table()[self.n_ctx:n_ctx]
                self.n_ctx = n_ctx
        nl = 0 if n_local is None or n_local >= n_ev else int(n_local)
        c = self.counts[slot].numpy()
        c[:] = records.counts_row(n_ev, n_sp, n_groups, nl, bases if self.wire == 16 and ev_pinned is not None
                                  else (t_base,), self.n_ctx if self.ctx is not None else 0, span_bytes)
        lab = self.labels[slot].numpy()
        lab[:] = -1
        if labels is not None:
            lab[: len(labels)] = labels
        self.k += 1
        dt = time.perf_counter() - t0
        self.encode_s += dt
        ctx = self.ctx is not None
        return StagedWindow(ev, sp, self.counts[slot], self.labels[slot], n_ev, n_sp, n_groups,
                            list(group_domains or []), self.wire, pod_table if self.wire == 32 else None,
                            self.ctx if ctx else None, self.n_ctx if ctx else 0, dt,
                            self.aux[slot] if self.aux is not None else None, span_bytes)


class WindowPipeline:
    def __init__(self, sig_cap: int, span_cap: int, group_cap: int, device: int = 0, process_group=None,
                 model: str = "bayes_learned", seed: int = 42, window_ms: float = 2000.0, threshold: float = 0.7,
                 fanout: int = 3, group_mode: int = 1, learn: bool = True, group_scope: str = "rank",
                 use_graphs: bool = True, max_ahead: int = 3, n_buffers: int = 3):
        import torch

        self.torch = torch
        self.dev = torch.device("cuda", device)
        self.pg = process_group
        self.model_name = model
        self.seed = seed
        self.learn = learn
        if group_scope not in ("rank", "global"):
            raise ValueError("group_scope must be 'rank' or 'global'")
        # "rank": incident groups are per-GPU (each node's services); "global": groups span
        # GPUs and are scored on all-reduced per-group sums (a second, G x 16 collective)
        self.group_scope = group_scope
        # learned naive Bayes refits on the device from accumulated all-reduced stats
        # (ops k_refit_nb): no per-window host round trip; LDA refits on the host
        self.device_refit = learn and model == "bayes_learned"
        # the per-window kernel chain (reset, decode, partition, join, finalize, posterior,
        # stats, pack: ~15 launches) is captured once per (buffer, shape) into a HIP graph
        # and replayed: window launch cost becomes one graph launch
        self.use_graphs = use_graphs
        self.graphs: Dict[tuple, object] = {}
        # host back-pressure: submit(i) first waits until window i - max_ahead has computed.
        # Stream-ordered waits alone let the host run arbitrarily far ahead; the runtime then
        # stalls the host for milliseconds at a time once its command queues fill
        # device input buffers: window i uses b = i % nb. With two, the H2D of window i waits
        # for window i-2's kernels, and the host (back-pressured on the same event) issues it
        # only after waking from that wait: the copy engine idled ~50 us per window. With three,
        # the H2D of window i depends on window i-3 and is queued before the engine frees up.
        self.nb = max(2, int(n_buffers))
        self.max_ahead = min(self.nb, max(1, int(max_ahead)))  # events exist for the last nb windows
        self.engine = GpuEngine(sig_cap, span_cap, group_cap, device, window_ms, threshold, fanout, group_mode)
        self.eng = self.engine.eng
        L = int(self.engine.mod.PACKET_LEN)
        if tuple(self.engine.mod.PACKET_LAYOUT) != PACKET_LAYOUT:
            raise RuntimeError("stale _mislo_hip build: packet layout mismatch (rebuild with ops.build)")
        self.packet_len = L
        with torch.cuda.device(self.dev):
            z8 = lambda n: torch.zeros(n, dtype=torch.uint8, device=self.dev)  # noqa: E731
            self.ev_dev = [z8(sig_cap * 64) for _ in range(self.nb)]
            # per buffer one [counts | labels | pad | spans] block (aux_head): a packed staged
            # window lands with a single H2D; the views keep fixed addresses for the graphs
            self.aux_head = aux_head(group_cap)
            self.aux_dev = [z8(self.aux_head + span_cap * 64) for _ in range(self.nb)]
            self.sp_dev = [a[self.aux_head:] for a in self.aux_dev]
            cb = 4 * records.COUNTS_LEN
            self.counts_dev = [a[:cb].view(torch.int32) for a in self.aux_dev]
            # append-only context table for 20-byte records: rows are copied once, stream
            # ordered before the first window that references them; the buffer address stays
            # fixed (captured graphs keep pointing at it) until it has to grow
            self.ctx_dev = torch.zeros((1 << 16, 4), dtype=torch.int32, device=self.dev)
            self.ctx_uploaded = 1  # row 0 = the all-zero context
            self.eng.set_ctx_table(self.ctx_dev)
            self.labels_dev = [a[cb:cb + 4 * max(group_cap, 1)].view(torch.int32) for a in self.aux_dev]
            for lab in self.labels_dev:
                lab.fill_(-1)
            self.packet_dev = [torch.zeros(L, dtype=torch.float64, device=self.dev) for _ in range(self.nb)]
            self.totals = torch.zeros(L, dtype=torch.float64, device=self.dev)
            self.host_s = [0.0, 0.0, 0.0, 0]
            self.stats_off = sum(PACKET_LAYOUT[:5])
            self.stats_acc = torch.zeros(PACKET_LAYOUT[5] + PACKET_LAYOUT[6], dtype=torch.float64, device=self.dev)
            p0 = np.zeros((16, 16), dtype=np.float64)
            p0[:, :N_DOMAINS] = NaiveBayes.random_init_table(seed)
            self.p0_dev = torch.from_numpy(p0.ravel()).to(self.dev)
            self.packet_host = [torch.zeros(L, dtype=torch.float64).pin_memory() for _ in range(self.nb)]
            # a model upload issued in submit(j) completes before window j+1 computes; the host
            # waits for window i - max_ahead, so max_ahead + 2 slots are never overwritten early
            self.model_host = [torch.zeros(2568, dtype=torch.uint8).pin_memory() for _ in range(self.max_ahead + 2)]
            self.copy_stream = torch.cuda.Stream(self.dev)
            self.comm_stream = torch.cuda.Stream(self.dev)
            self.compute_stream = torch.cuda.Stream(self.dev)
            ev = lambda: torch.cuda.Event()  # noqa: E731
            self.h2d_done = [ev() for _ in range(self.nb)]
            self.compute_done = [ev() for _ in range(self.nb)]
            self.comm_done = [ev() for _ in range(self.nb)]
            self.join_done, self.groups_done = ev(), ev()
        self.pod_key = None
        self.i = 0
        self.cum_stats = SufficientStats()
        self.windows_folded = 0
        self.model = self._initial_model()
        self._upload_model(self.model)
        self.last_refit_s = 0.0

    # ---------------------------------------------------------------------------------
    def _initial_model(self):
        if self.model_name == "bayes":
            return NaiveBayes.ref()
        if self.model_name == "lda":
            return NaiveBayes.learned(SufficientStats(), seed=self.seed)  # until stats exist
        return NaiveBayes.learned(SufficientStats(), seed=self.seed)

    def _upload_model(self, model) -> None:
        torch = self.torch
        slot = self.i % len(self.model_host)
        host = self.model_host[slot]
        host.numpy()[:] = model_bytes(model)
        with torch.cuda.stream(self.compute_stream):
            self.eng.set_model_bytes(host)

    def refit(self, stats: SufficientStats) -> None:
        t = time.perf_counter()
        if self.model_name == "lda" and stats.count.sum() > 32:
            self.model = LDA.fit(stats)
        elif self.model_name in ("bayes_learned", "lda"):
            self.model = NaiveBayes.learned(stats, seed=self.seed)
        self._upload_model(self.model)
        self.last_refit_s = time.perf_counter() - t

    # ---------------------------------------------------------------------------------
    def submit(self, w: StagedWindow, with_labels: bool = True) -> None:
        t_enter = time.perf_counter()
        torch = self.torch
        b = self.i % self.nb
        cs, ks, ms = self.copy_stream, self.compute_stream, self.comm_stream
        if self.i >= self.max_ahead:
            self.compute_done[(self.i - self.max_ahead) % self.nb].synchronize()
        # H2D into buffer b once window i-nb (the last user of b) finished computing
        cs.wait_event(self.compute_done[b])
        if w.pod_table is not None:
            key = (w.pod_table.shape[0], hash(w.pod_table.tobytes()))
            if key != self.pod_key:  # interned pod table changed: re-upload (rare)
                self.drain()
                self.engine.set_pod_table(w.pod_table)
                self.pod_key = key
                self.graphs = {}  # captured launches hold the old table's address
        if w.n_ctx > self.ctx_dev.shape[0]:  # grow the context table (rare): re-capture
            self.drain()
            cap = 1 << int(np.ceil(np.log2(w.n_ctx)))
            grown = torch.zeros((cap, 4), dtype=torch.int32, device=self.dev)
            grown[: self.ctx_uploaded].copy_(self.ctx_dev[: self.ctx_uploaded])
            self.ctx_dev = grown
            self.eng.set_ctx_table(self.ctx_dev)
            self.graphs = {}
        tr = [time.perf_counter()] if _HOST_TRACE else None
        with torch.cuda.stream(cs):
            if w.n_ctx > self.ctx_uploaded:  # new context rows (append-only ids)
                self.ctx_dev[self.ctx_uploaded: w.n_ctx].copy_(w.ctx_rows[self.ctx_uploaded: w.n_ctx],
                                                               non_blocking=True)
                self.ctx_uploaded = w.n_ctx
            nb = w.n_events * records.wire_bytes(w.wire)
            self.ev_dev[b][:nb].copy_(w.ev[:nb], non_blocking=True)
            if tr: tr.append(time.perf_counter())
            if w.aux is not None and w.aux.numel() >= self.aux_head and \
                    w.counts.data_ptr() == w.aux.data_ptr() and w.sp.data_ptr() == w.aux.data_ptr() + self.aux_head:
                # packed block: counts, labels and spans in one DMA (a copy has a fixed
                # ~10 us cost on the copy engine, paid per window on the critical path)
                na = self.aux_head + w.n_spans * w.span_bytes
                self.aux_dev[b][:na].copy_(w.aux[:na], non_blocking=True)
                if tr: tr.extend([time.perf_counter()] * 3)
            else:
                self.sp_dev[b][: w.n_spans * w.span_bytes].copy_(w.sp[: w.n_spans * w.span_bytes], non_blocking=True)
                if tr: tr.append(time.perf_counter())
                self.counts_dev[b].copy_(w.counts, non_blocking=True)
                if tr: tr.append(time.perf_counter())
                self.labels_dev[b].copy_(w.labels, non_blocking=True)
                if tr: tr.append(time.perf_counter())
            self.h2d_done[b].record(cs)
        if tr:
            tr.append(time.perf_counter())
            print("[host-trace] pre %.1f ev %.1f sp %.1f counts %.1f labels %.1f record %.1f us" % (
                1e6 * (tr[0] - t_enter), *(1e6 * (tr[j + 1] - tr[j]) for j in range(5))), flush=True)
        t_copy = time.perf_counter()
        ks.wait_event(self.h2d_done[b])
        ks.wait_event(self.comm_done[b])  # packet[b] no longer being reduced / read
        with torch.cuda.stream(ks):
            if self.device_refit and self.i >= self.nb:
                # fold window i-nb's all-reduced statistics (packet[b], complete per the wait
                # above) and refit before window i: deterministic prequential lag of nb
                n = self.stats_acc.numel()
                self.eng.refit_nb(self.stats_acc, self.p0_dev, 2.0, 1.0, N_DOMAINS,
                                  self.packet_dev[b][self.stats_off:self.stats_off + n])
                self.windows_folded += 1
            self.eng.bind_io(self.counts_dev[b], self.labels_dev[b], self.packet_dev[b])
            if self.group_scope == "global" and self.pg is not None:
                self.eng.run_window_pre(self.ev_dev[b], self.sp_dev[b], w.n_groups, w.wire)
                self.join_done.record(ks)
        if self.group_scope == "global" and self.pg is not None:
            # group sums of this window across the node, then posterior on the global features
            ms.wait_event(self.join_done)
            with torch.cuda.stream(ms):
                torch.distributed.all_reduce(self.eng.gsum[: w.n_groups], group=self.pg)
                torch.distributed.all_reduce(self.eng.gcnt[: w.n_groups], group=self.pg)
                self.groups_done.record(ms)
            ks.wait_event(self.groups_done)
            with torch.cuda.stream(ks):
                self.eng.run_window_post(w.n_groups, with_labels, self.learn and with_labels)
                self.compute_done[b].record(ks)
        else:
            with torch.cuda.stream(ks):
                self._run_window(b, w, with_labels)
                self.compute_done[b].record(ks)
        t_compute = time.perf_counter()
        ms.wait_event(self.compute_done[b])
        with torch.cuda.stream(ms):
            if self.pg is not None:
                torch.distributed.all_reduce(self.packet_dev[b], group=self.pg)
            self.totals.add_(self.packet_dev[b])
            self.packet_host[b].copy_(self.packet_dev[b], non_blocking=True)
            self.comm_done[b].record(ms)
        t_exit = time.perf_counter()
        hs = self.host_s  # host time spent issuing: copies / compute / comm
        hs[0] += t_copy - t_enter
        hs[1] += t_compute - t_copy
        hs[2] += t_exit - t_compute
        hs[3] += 1
        self.i += 1
        # fold window i-2 (this call's predecessor's predecessor is certainly far along;
        # folding i-1 would stall the host on the window just queued)
        if self.i >= 2 and self.learn and not self.device_refit:
            pb = (self.i - 2) % self.nb
            self.comm_done[pb].synchronize()
            pk = unpack_packet(self.packet_host[pb].numpy())
            self.cum_stats = self.cum_stats.merge(stats_from_packet(pk))
            self.windows_folded += 1
            self.refit(self.cum_stats)

    def _run_window(self, b: int, w: StagedWindow, with_labels: bool) -> None:
        learn = self.learn and with_labels
        args = (self.ev_dev[b], self.sp_dev[b], w.n_groups, with_labels, learn, w.wire)
        if not self.use_graphs:
            self.eng.run_window(*args)
            return
        torch = self.torch
        key = (b, w.n_groups, with_labels, learn, w.wire)
        g = self.graphs.get(key)
        if g is None:
            if not self.graphs.get(("warm", b)):  # first use of the buffers: run eagerly once
                self.eng.run_window(*args)
                self.graphs[("warm", b)] = True
                return
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=torch.cuda.current_stream(self.dev), capture_error_mode="thread_local"):
                self.eng.run_window(*args)
            self.graphs[key] = g
        g.replay()

    def host_model(self):
        """The model currently on the device, as a host LinearPosteriorModel (reporting)."""
        if not self.device_refit:
            return self.model
        self.drain()
        st = self.stats_acc.cpu().numpy()
        s = SufficientStats(count=st[1024:1024 + N_DOMAINS].copy(),
                            elevated_sum=st[:1024].reshape(32, 32)[:16, :N_DOMAINS].copy(),
                            x_sum=st[:1024].reshape(32, 32)[16:, :N_DOMAINS].copy(),
                            xx=st[:1024].reshape(32, 32)[16:, 16:].copy())
        self.model = NaiveBayes.learned(s, seed=self.seed)
        return self.model

    def last_packet(self) -> Dict[str, np.ndarray]:
        """Unpacked (all-reduced) packet of the most recently submitted window (after drain)."""
        b = (self.i - 1) % self.nb
        self.comm_done[b].synchronize()
        return unpack_packet(self.packet_host[b].numpy().copy())

    def drain(self) -> None:
        self.torch.cuda.synchronize(self.dev)

    def reset_totals(self) -> None:
        self.drain()
        self.totals.zero_()
        self.host_s = [0.0, 0.0, 0.0, 0]

    def host_issue_us(self) -> Dict[str, float]:
        """Mean host time per submitted window spent issuing each stream's work (us)."""
        n = max(self.host_s[3], 1)
        return {"copy": 1e6 * self.host_s[0] / n, "compute": 1e6 * self.host_s[1] / n,
                "comm": 1e6 * self.host_s[2] / n}

    def summary(self) -> Dict[str, object]:
        self.drain()
        p = unpack_packet(self.totals.cpu().numpy())
        conf = p["confusion"][:N_DOMAINS, :N_DOMAINS].astype(np.int64)
        return {
            "confusion": conf,
            "macro_f1": macro_f1_from_confusion(conf),
            "accuracy": float(np.trace(conf) / conf.sum()) if conf.sum() else 0.0,
            "hist": p["hist"].astype(np.int64),
            "status": p["status"].astype(np.int64),
            "dbg": p["dbg"].astype(np.int64),
            "misc": p["misc"].astype(np.int64),
            "stats": stats_from_packet(p),
        }
