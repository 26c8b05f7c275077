"""Per-GPU window pipeline: the agent's window sources feeding the native window engine.

The per-window path has no Python per event and no PyTorch at all:

* a window SOURCE closes the window (publishes the next epoch into ``mislo_cfg``, snapshots the
  ring positions: the cut) and its native ``WindowAssembler`` (runtime/csrc/assemble.h)
  compacts the BPF ring's EVENT16 records up to the cut into the pinned input block of the
  window's engine buffer, applies the probes' id definitions, encodes user-space producers'
  64-byte records and the window's spans, and writes the context-row patch and the counts;
* the native ``WindowEngine`` (ops/csrc/engine.h) DMAs the block in one copy and replays the
  buffer's captured HIP graph (decode -> LDS join -> MFMA posterior/statistics -> pack) on the
  compute stream, while the RCCL all-reduce of the previous window's packed statistics runs on
  the comm stream; the learned model refits on the device (prequential, lag = buffers).

``WindowPipeline`` is the Python handle on the engine (model upload, totals, results);
``RingWindowSource`` is the kernel-ring source (a pinned BPF ring buffer map, or the
shared-memory emulation tests and the benchmark use); ``build_replay_images`` turns seeded
fault-replay windows into the bytes the probes would have written (native probe model).
"""

from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from ..collector import records
from ..models.bayes import LDA, N_DOMAINS, NaiveBayes, SufficientStats
from ..models.metrics import macro_f1_from_confusion

PACKET_LAYOUT = (256, 48, 18, 8, 256, 1024, 16)  # hist, status, misc(+16 value sums), dbg, confusion, stats, count
ROW_CAP = 1 << 17


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


def summarize(p: np.ndarray) -> Dict[str, object]:
    u = unpack_packet(p)
    conf = u["confusion"][:N_DOMAINS, :N_DOMAINS].astype(np.int64)
    return {
        "confusion": conf,
        "macro_f1": macro_f1_from_confusion(conf),
        "accuracy": float(np.trace(conf) / conf.sum()) if conf.sum() else 0.0,
        "hist": u["hist"].astype(np.int64),
        "status": u["status"].astype(np.int64),
        "dbg": u["dbg"].astype(np.int64),
        "misc": u["misc"].astype(np.int64),
        "stats": stats_from_packet(u),
    }


class WindowPipeline:
    """Python handle on one native WindowEngine (one MI355X). ``comm`` = (unique_id bytes,
    rank, world) joins the node's RCCL communicator for the per-window packet all-reduce."""

    def __init__(self, sig_cap: int, span_cap: int, group_cap: int, device: int = 0, comm=None,
                 model: str = "bayes_learned", seed: int = 42, window_ms: float = 2000.0, threshold: float = 0.7,
                 fanout: int = 3, group_mode: int = 1, learn: bool = True, use_graphs: bool = True,
                 max_ahead: int = 3, n_buffers: int = 3, row_cap: int = ROW_CAP):
        from ..ops import load_agent
        from ..ops.engine import model_bytes

        self.mod = load_agent()
        if tuple(self.mod.PACKET_LAYOUT) != PACKET_LAYOUT:
            raise RuntimeError("stale _mislo_agent build: packet layout mismatch (rebuild with ops.build)")
        self.model_name, self.seed, self.learn = model, seed, learn
        self.device_refit = learn and model == "bayes_learned"
        self._model_bytes = model_bytes
        self.eng = self.mod.WindowEngine(device=device, sig_cap=sig_cap, span_cap=span_cap, group_cap=group_cap,
                                         row_cap=row_cap, n_buffers=n_buffers, max_ahead=max_ahead,
                                         window_ms=window_ms, threshold=threshold, fanout=fanout,
                                         group_mode=group_mode, use_graphs=use_graphs,
                                         device_refit=self.device_refit, n_dom=N_DOMAINS)
        self.nb = self.eng.buffers
        self.layout = self.eng.layout
        self.sig_cap, self.span_cap, self.group_cap, self.row_cap = sig_cap, span_cap, group_cap, row_cap
        if comm is not None and comm[2] > 1:
            self.eng.init_comm(comm[0], comm[1], comm[2])
        p0 = np.zeros((16, 16), dtype=np.float64)
        p0[:, :N_DOMAINS] = NaiveBayes.random_init_table(seed)
        self.eng.set_p0(p0.ravel())
        self.cum_stats = SufficientStats()
        self.model = self._initial_model()
        self.eng.set_model_bytes(model_bytes(self.model))
        self.k = 0
        self.windows_folded_host = 0

    def _initial_model(self):
        if self.model_name == "bayes":
            return NaiveBayes.ref()
        return NaiveBayes.learned(SufficientStats(), seed=self.seed)

    # ---- per window -----------------------------------------------------------------------
    def slot(self, k: Optional[int] = None) -> int:
        """Address of the pinned input block of window ``k`` (default: the next one), after
        waiting until its previous reader's DMA is done."""
        k = self.k if k is None else k
        self.eng.wait_slot(k)
        return self.eng.host_slot(k)

    def submit(self, dma_bytes: int, n_groups: int, with_labels: bool = True, learn: Optional[bool] = None) -> int:
        k = self.k
        learn = (self.learn and with_labels) if learn is None else learn
        self.eng.submit(k, int(dma_bytes), int(n_groups), bool(with_labels), bool(learn))
        self.k += 1
        if self.learn and not self.device_refit and k >= 2:
            self._host_refit(k - 2)  # window k-2 is done or nearly (k-1 would stall the host)
        return k

    def _host_refit(self, j: int) -> None:
        """LDA (or host-refit Bayes): fold window j's all-reduced statistics on the host."""
        self.eng.wait(j)
        pk = unpack_packet(self.eng.packet(j))
        self.cum_stats = self.cum_stats.merge(stats_from_packet(pk))
        self.windows_folded_host += 1
        if self.model_name == "lda" and self.cum_stats.count.sum() > 32:
            self.model = LDA.fit(self.cum_stats)
        elif self.model_name in ("bayes_learned", "lda"):
            self.model = NaiveBayes.learned(self.cum_stats, seed=self.seed)
        self.eng.set_model_bytes(self._model_bytes(self.model))

    def wait(self, k: int) -> None:
        self.eng.wait(k)

    def packet(self, k: int) -> Dict[str, np.ndarray]:
        self.eng.wait(k)
        return unpack_packet(self.eng.packet(k))

    def results(self, k: int, n_groups: int) -> Dict[str, np.ndarray]:
        self.eng.wait(k)
        return self.eng.results(k, n_groups)

    def window_ms(self, k: int):
        return self.eng.window_ms(k)

    def set_model(self, model) -> None:
        self.model = model
        self.eng.set_model_bytes(self._model_bytes(model))

    # ---- totals / model ---------------------------------------------------------------------
    def drain(self) -> None:
        self.eng.sync()

    def reset_totals(self) -> None:
        self.eng.reset_totals()

    @property
    def windows_folded(self) -> int:
        return int(self.eng.windows_folded) + self.windows_folded_host

    def summary(self) -> Dict[str, object]:
        return summarize(self.eng.totals())

    def host_model(self):
        """The model currently on the device, as a host LinearPosteriorModel (reporting)."""
        if not self.device_refit:
            return self.model
        st = self.eng.stats_acc()
        s = SufficientStats(count=st[1024:1024 + N_DOMAINS].copy(),
                            elevated_sum=st[:1024].reshape(32, 32)[:16, :N_DOMAINS].copy(),
                            x_sum=st[:1024].reshape(32, 32)[16:, :N_DOMAINS].copy(),
                            xx=st[:1024].reshape(32, 32)[16:, 16:].copy())
        return NaiveBayes.learned(s, seed=self.seed)


# ---------------------------------------------------------------------------------------
# window sources
# ---------------------------------------------------------------------------------------

@dataclass
class Cut:
    """A window boundary: ring positions to consume up to and the 4 epoch bases by tag."""
    kernel: int = (1 << 64) - 1
    user: int = (1 << 64) - 1
    spans: int = (1 << 64) - 1
    bases: Sequence[int] = (0, 0, 0, 0)
    t_ns: int = 0


class RingWindowSource:
    """Kernel-ring window source: consumes the BPF ring buffer (``ring``: a pinned map opened
    with Ringbuf.open_pinned, or an emulated one), optional user-space event and span rings,
    through the native tables and assembler into a WindowPipeline's input blocks.

    ``cut()`` is the live protocol (the agent is the clock): publish epoch k into mislo_cfg
    (``cfg_set``: the emulated array, or the real map's BpfMap update), then snapshot every
    ring's producer position; records a probe stamps from then on carry the new tag, records
    stamped before it keep theirs and decode against the bases the window ships."""

    def __init__(self, pipe: WindowPipeline, ring=None, user_ring=None, span_ring=None, threads: int = 8,
                 cfg_set=None, tables=None):
        from ..runtime import load

        self.rt = load()
        self.pipe = pipe
        self.ring, self.user_ring, self.span_ring = ring, user_ring, span_ring
        self.tables = tables if tables is not None else records.native_tables()
        self.consumer = self.rt.RingbufConsumer(ring, threads) if ring is not None else None
        L = pipe.layout
        self.asm = self.rt.WindowAssembler(pipe.group_cap, pipe.span_cap, pipe.sig_cap, pipe.row_cap, self.tables,
                                           self.consumer, user_ring, span_ring)
        self.clock = records.EpochClock()
        if cfg_set is None and ring is not None and getattr(ring, "emulated", False):
            cfg_set = lambda i, v: ring.cfg_set(i, v)  # noqa: E731
        self.cfg_set = cfg_set
        self.last: Dict[str, object] = {}
        self.host_s = 0.0
        self.n = 0
        assert L["ev_off"] > 0

    def publish_epoch(self, now_ns: Optional[int] = None) -> int:
        v = self.clock.publish(int(now_ns if now_ns is not None else time.time_ns()))
        if self.cfg_set is not None:
            self.cfg_set(self.rt.CFG_EPOCH, v)
        return v

    def cut(self, now_ns: Optional[int] = None) -> Cut:
        """Close the window at ``now_ns``: new epoch first, then the ring snapshots."""
        t = int(now_ns if now_ns is not None else time.time_ns())
        self.publish_epoch(t)
        return Cut(kernel=self.ring.producer_pos if self.ring is not None else 0,
                   user=self.user_ring.head if self.user_ring is not None else 0,
                   spans=self.span_ring.head if self.span_ring is not None else 0,
                   bases=self.clock.bases(), t_ns=t)

    def stage(self, cut: Cut, n_groups: int, labels: Optional[np.ndarray] = None) -> Dict[str, object]:
        """Assemble the window up to ``cut`` into the pipeline's next input block."""
        t0 = time.perf_counter()
        slot = self.pipe.slot()
        r = self.asm.assemble(slot, list(cut.bases), n_groups, labels, cut.kernel, cut.user, cut.spans)
        self.host_s += time.perf_counter() - t0
        self.n += 1
        self.last = r
        return r

    def group_sli(self) -> np.ndarray:
        """[group_cap, 2] spans and TTFT-SLO breaches per incident group since the last call."""
        return self.tables.take_group_sli(self.pipe.group_cap).astype(np.float64)

    def step(self, n_groups: int, labels=None, cut: Optional[Cut] = None, with_labels: Optional[bool] = None) -> int:
        """cut (live, unless given) -> assemble -> submit; returns the window index."""
        c = cut if cut is not None else self.cut()
        r = self.stage(c, n_groups, labels)
        wl = labels is not None if with_labels is None else with_labels
        return self.pipe.submit(r["dma_bytes"], n_groups, with_labels=wl)


@dataclass
class ReplayImage:
    """A fault-replay window as the probes would have written it: framed ring bytes (events +
    definitions, epoch-stamped against ``bases``), spans and user-space records, labels."""
    framed: np.ndarray
    spans: np.ndarray
    user: np.ndarray
    bases: tuple
    n_groups: int
    labels: np.ndarray
    domains: List[List[str]] = field(default_factory=list)
    n_kernel: int = 0


def kernel_event_mask(events: np.ndarray) -> np.ndarray:
    """Which replay events the kernel probes emit (CPU/network/scheduler/memory/disk signals);
    the rest (the 4 GPU signals) come from the rocprofiler-sdk tool's user-space ring."""
    from ..signals import catalog

    gpu_types = np.array([s.kernel_type for s in catalog.SIGNALS if s.name in catalog.GPU_SIGNALS], dtype=np.uint16)
    return ~np.isin(events["signal_type"], gpu_types)


def build_replay_images(windows, shift=None, window_ns: int = 1_000_000_000, sim_ring=None) -> List[ReplayImage]:
    """Run replay windows through the native probe model (one epoch per window cut, published
    at the window start): kernel-signal events become framed EVENT16 ring bytes, GPU-signal
    events stay 64-byte user-space records, spans stay 64-byte span records."""
    from ..runtime import load

    rt = load()
    shift = records.milli_shift_table() if shift is None else shift
    own = sim_ring is None
    if own:
        sim_ring = rt.Ringbuf.create_shm(f"/mislo-sim-{os.getpid()}-{id(windows)}", 1 << 16)
    sim = rt.ProbeSim(sim_ring, shift)
    clock = records.EpochClock()
    out = []
    for i, w in enumerate(windows):
        if i == 0:  # the epoch in force before the first window
            sim_ring.cfg_set(rt.CFG_EPOCH, clock.publish(int(w.t0_ns) - window_ns))
        km = kernel_event_mask(w.events)
        kev = np.ascontiguousarray(w.events[km])
        # records stamped before the cut carry the previous epoch's tag (late writers across the
        # cut), the rest the epoch the agent published at the window start
        early = (kev["ts_ns"] < int(w.t0_ns)) & (kev["ts_ns"] != 0)
        parts = [sim.encode(np.ascontiguousarray(kev[early]))]
        sim_ring.cfg_set(rt.CFG_EPOCH, clock.publish(int(w.t0_ns)))
        parts.append(sim.encode(np.ascontiguousarray(kev[~early])))
        payload = np.concatenate(parts)
        out.append(ReplayImage(framed=rt.frame_records(payload), spans=np.ascontiguousarray(w.spans),
                               user=np.ascontiguousarray(w.events[~km]), bases=clock.bases(), n_groups=w.n_groups,
                               labels=np.asarray(w.group_labels, dtype=np.int32), domains=list(w.group_domains),
                               n_kernel=int(km.sum())))
    return out
