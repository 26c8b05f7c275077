"""Per-GPU window pipeline: the agent's rings feeding the native window engine, zero-copy.

The agent's CPU never reads, rewrites or re-encodes a record:

* the window SOURCE closes a window (publishes the next epoch into ``mislo_cfg``, then
  snapshots the rings' producer positions: the cut) and hands the engine byte RANGES: the BPF
  ring buffer's framed records since the last cut (one contiguous range thanks to the ring's
  double mapping), the user-space producers' 64-byte records and the spans (<= 2 ranges each);
* the native ``WindowEngine`` (ops/csrc/engine.h) DMAs those ranges straight from the
  page-locked rings into HBM and replays the buffer's captured HIP graph: ring definitions
  (context rows, trace map) -> decode of framed + user records -> LDS join -> MFMA
  posterior/statistics -> pack, while the RCCL all-reduce of the previous window's packed
  statistics runs on the comm stream; the learned model refits on the device (prequential);
* ring space is freed once the DMA that read it has completed (user / span rings) or once
  the window's results say no record in it was still being written (the BPF ring: a record
  the GPU found busy is re-submitted with the next window, exactly once).

``WindowPipeline`` is the Python handle on the engine (model upload, totals, results);
``RingWindowSource`` the ring source (a pinned BPF ring buffer map, or the shared-memory
emulation tests and the benchmark use); ``build_replay_images`` turns seeded fault-replay
windows into the bytes the probes would have written (native probe model).
"""

from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..collector import records
from ..models.bayes import LDA, N_DOMAINS, NaiveBayes, SufficientStats
from ..models.metrics import macro_f1_from_confusion
from ..signals import catalog

# hist, status, misc(+16 value sums), dbg, confusion, stats, count, ring accounting
PACKET_LAYOUT = (256, 48, 18, 8, 256, 1024, 16, 8)
RS, BS = records.REC_STRIDE, records.BATCH_SLOTS  # BPF ring: bytes per batch record, rows (slots) per record
RING_FIELDS = ("first_busy", "foreign", "def_ctx", "def_trace", "discarded", "events", "other_shard")
USER_CAP = 1 << 18


def unpack_packet(p: np.ndarray) -> Dict[str, np.ndarray]:
    o = 0
    out = {}
    for name, n in zip(("hist", "status", "misc", "dbg", "confusion", "stats", "count", "ring"), PACKET_LAYOUT):
        out[name] = p[o:o + n]
        o += n
    out["hist"] = out["hist"].reshape(16, 16)
    out["status"] = out["status"].reshape(16, 3)
    out["confusion"] = out["confusion"].reshape(16, 16)
    out["stats"] = out["stats"].reshape(32, 32)
    out["value_sum"] = out["misc"][2:18] * 1e-3  # per-slot sums of decoded values (output units)
    out["ring_state"] = {k: int(v) for k, v in zip(RING_FIELDS, out["ring"][:len(RING_FIELDS)])}
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
        "ring": u["ring"].astype(np.int64),
        "stats": stats_from_packet(u),
    }


class WindowPipeline:
    """Python handle on one native WindowEngine (one MI355X). ``comm`` = (unique_id bytes,
    rank, world) joins the node's RCCL communicator: per window, the packet all-reduce, the
    all-gather of every GPU's incident results and (``xchg_cap``) of the trace-tagged rows
    each GPU imports into its window. ``halo_ms``: later windows also join a window's rows within
    that distance of every later window's latest record (joins across the cut); the rows of
    ``halo_windows`` earlier windows stay resident on the device for it. ``import_cap`` bounds
    the other GPUs' rows per window."""

    def __init__(self, sig_cap: int, span_cap: int, group_cap: int, device: int = 0, comm=None,
                 model: str = "bayes_learned", seed: int = 42, window_ms: float = 2000.0, threshold: float = 0.7,
                 fanout: int = 3, group_mode: int = 1, learn: bool = True, use_graphs: bool = True,
                 max_ahead: int = 3, n_buffers: int = 3, user_cap: int = USER_CAP, ttft_slo_ms: float = 800.0,
                 halo_ms: float = 0.0, import_cap: int = 0, xchg_cap: int = 0, shard: Tuple[int, int] = (0, 1),
                 engine: str = "gpu", group=None, model_image: Optional[np.ndarray] = None, halo_windows: int = 3,
                 split_rings: bool = False):
        """``engine``: "gpu" = the native WindowEngine on HIP device ``device`` (``comm`` = its RCCL
        communicator); "cpu" = pipeline.cpu.CpuRingEngine, the same contract on the host, with
        ``group`` (a torch.distributed gloo group) as its communicator. ``shard`` = (rank, world):
        this engine's share of one node's stream (group sharding, decode.hip shard_owns);
        ``split_rings``: the records arrive already routed to this worker's own rings (no record
        ownership filter; spans keep theirs).
        ``model_image``: a PosteriorModel image to score with (models/export.py) instead of ``model``'s
        built-in initial model."""
        from ..ops.engine import model_bytes

        self.model_name, self.seed, self.learn = model, seed, learn
        self.device_refit = learn and model == "bayes_learned" and engine == "gpu" and model_image is None
        self._model_bytes = model_bytes
        user_cap = max(1, min(int(user_cap), int(sig_cap)))
        kw = dict(device=device, sig_cap=sig_cap, span_cap=span_cap, group_cap=group_cap, user_cap=user_cap,
                  n_buffers=n_buffers, window_ms=window_ms, threshold=threshold, fanout=fanout, group_mode=group_mode,
                  n_dom=N_DOMAINS, ttft_slo_ms=ttft_slo_ms, halo_ms=halo_ms, import_cap=import_cap, xchg_cap=xchg_cap,
                  shard_rank=int(shard[0]), shard_world=int(shard[1]), halo_windows=int(halo_windows),
                  split_rings=bool(split_rings))
        self.engine_kind = engine
        if engine == "cpu":
            from .cpu import CpuRingEngine

            self.mod = None
            self.stats_off, self.stats_len = sum(PACKET_LAYOUT[:5]), PACKET_LAYOUT[5] + PACKET_LAYOUT[6]
            self.eng = CpuRingEngine(group=group, **kw)
        elif engine == "gpu":
            from ..ops import load_agent

            self.mod = load_agent()
            if tuple(self.mod.PACKET_LAYOUT) != PACKET_LAYOUT:
                raise RuntimeError("stale _mislo_agent build: packet layout mismatch (rebuild with ops.build)")
            self.stats_off, self.stats_len = int(self.mod.STATS_OFF), int(self.mod.STATS_LEN)
            if os.environ.get("MISLO_GRAPHS", "") == "0":  # diagnostic: plain launches instead of HIP graphs
                use_graphs = False
            self.eng = self.mod.WindowEngine(max_ahead=max_ahead, use_graphs=use_graphs,
                                             device_refit=self.device_refit, **kw)
        else:
            raise ValueError(f"unknown window engine {engine!r} (gpu | cpu)")
        self.halo_ms, self.import_cap, self.xchg_cap = halo_ms, import_cap, xchg_cap
        self.shard = (int(shard[0]), int(shard[1]))
        self.nb = self.eng.buffers
        self.sig_cap, self.span_cap, self.group_cap, self.user_cap = sig_cap, span_cap, group_cap, user_cap
        if comm is not None and comm[2] >= 1:  # (uid, rank, world); world 1 = a one-rank communicator
            self.eng.init_comm(comm[0], comm[1], comm[2])
        p0 = np.zeros((16, 16), dtype=np.float64)
        p0[:, :N_DOMAINS] = NaiveBayes.random_init_table(seed)
        self.eng.set_p0(p0.ravel())
        # NaiveBayes.learned's arguments the device refit mirrors (set_prior changes them)
        self.learned_kw: Dict[str, object] = {"seed": seed}
        self.cum_stats = SufficientStats()
        if model_image is not None:
            from ..ops.engine import model_from_bytes

            self.model = model_from_bytes(model_image)
            self.eng.set_model_bytes(np.ascontiguousarray(model_image, dtype=np.uint8))
        else:
            self.model = self._initial_model()
            self.eng.set_model_bytes(model_bytes(self.model))
        self.k = 0
        self.windows_folded_host = 0

    def _initial_model(self):
        if self.model_name == "bayes":
            return NaiveBayes.ref()
        if self.model_name == "bayes_gpu":
            return NaiveBayes.gpu()
        return NaiveBayes.learned(SufficientStats(), seed=self.seed)

    def set_prior(self, init: Optional[np.ndarray] = None, floor: Optional[np.ndarray] = None,
                  cap_domain: Optional[str] = None, ceil: Optional[float] = None) -> None:
        """The learned model's Beta prior table [16, D] (None: the seeded random-init one), its
        likelihood floor [16, D] and the capped-prior domain (models/train.py learned_kwargs), on
        the device refit (k_refit_nb) and the host mirror alike; ``ceil`` caps every likelihood
        (the device's through set_refit, ``lik_ceil()``). The refit's other parameters stay
        set_refit's."""
        p0 = np.zeros((2, 16, 16), dtype=np.float64)
        p0[0, :, :N_DOMAINS] = init if init is not None else NaiveBayes.random_init_table(self.seed)
        if floor is not None:
            p0[1, :, :N_DOMAINS] = floor
        self.eng.set_p0(p0.ravel())
        self.learned_kw = {"seed": self.seed, "init": init, "floor": floor, "cap_domain": cap_domain, "ceil": ceil}

    def lik_ceil(self) -> float:
        """The likelihood cap for set_refit (1.0: none)."""
        c = self.learned_kw.get("ceil")
        return 1.0 if c is None else float(c)

    def cap_dom(self) -> int:
        """The capped-prior domain's index for set_refit (-1: none)."""
        c = self.learned_kw.get("cap_domain")
        return -1 if c is None else catalog.DOMAIN_INDEX[str(c)]

    # ---- per window -----------------------------------------------------------------------
    def submit(self, kernel, user, spans, n_groups: int, labels=None, bases=(0, 0, 0, 0), with_labels: bool = True,
               learn: Optional[bool] = None, user_rec: int = 64) -> int:
        """Queue the next window: ``kernel`` / ``user`` / ``spans`` = [(host address, bytes)] ranges
        of framed ring records / ``user_rec``-byte records / 64-byte spans. Returns its index.
        USER24 records (``user_rec`` 24) keep 44 timestamp bits, resolved against the newest of
        ``bases``: a window of them needs a published epoch."""
        if user_rec in (16, 24) and not any(int(b) for b in bases) and any(int(n) for _, n in user):
            raise ValueError("USER24 records need the window's epoch bases (all are 0)")
        k = self.k
        learn = (self.learn and with_labels) if learn is None else learn
        lab = None if labels is None else np.ascontiguousarray(labels, dtype=np.int32)
        self.eng.submit(k, list(kernel), list(user), list(spans), int(n_groups), lab, [int(b) for b in bases],
                        bool(with_labels), bool(learn), int(user_rec))
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
            self.model = NaiveBayes.learned(self.cum_stats, **self.learned_kw)
        self.model.app = getattr(self, "app", None)
        self.eng.set_model_bytes(self._model_bytes(self.model))

    def wait(self, k: int) -> None:
        self.eng.wait(k)

    def packet(self, k: int) -> Dict[str, np.ndarray]:
        self.eng.wait(k)
        return unpack_packet(self.eng.packet(k))

    def results(self, k: int, n_groups: int) -> Dict[str, np.ndarray]:
        self.eng.wait(k)
        return self.eng.results(k, n_groups)

    def results_all(self, k: int, n_groups: int) -> List[Dict[str, np.ndarray]]:
        """Every GPU's incident results of window k (RCCL all-gather; this GPU's alone when the
        node has one): the node-wide incident list."""
        self.eng.wait(k)
        return self.eng.results_all(k, n_groups)

    def inject_remote(self, blocks: np.ndarray, world: int, me: int) -> None:
        """Rows for the next window as other GPUs' exchange blocks deliver them (oracle.exchange_blocks)."""
        self.eng.inject_remote(np.ascontiguousarray(blocks, dtype=np.uint8), len(blocks) // world, world, me)

    def window_ms(self, k: int):
        return self.eng.window_ms(k)

    def set_model(self, model) -> None:
        self.model = model
        self.eng.set_model_bytes(self._model_bytes(model))
        if getattr(self, "app", None) is not None and model.app is None:
            model.app = self.app
        if model.app is not None:
            self.set_app(model.app)

    def set_app(self, app) -> None:
        """The application evidence (models/bayes.py AppEvidence; None: off) the posterior kernel
        adds to every incident group whose spans report a retrieval time. Its 2-fault columns
        follow the current model's pairs."""
        from ..ops.engine import app_model_bytes

        self.app = app
        self.model.app = app
        self.eng.set_app_model(app_model_bytes(self.model))

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

    # ---- checkpoint / resume (utils/checkpoint.py) ------------------------------------------
    def state(self) -> Tuple[Dict[str, np.ndarray], Dict[str, object]]:
        """Everything the learned model depends on (arrays, metadata); drains the engine. The
        device refit runs nb windows behind: the statistics of the windows it has not folded
        yet (their all-reduced packets) are added, so the checkpoint holds every finished
        window (the restored engine refits from them)."""
        self.drain()
        c = self.cum_stats
        stats = np.asarray(self.eng.stats_acc(), dtype=np.float64).copy()
        off, n = self.stats_off, self.stats_len
        pending = range(max(0, self.k - self.nb), self.k) if self.device_refit else range(0)
        for j in pending:
            stats += np.asarray(self.eng.packet(j), dtype=np.float64)[off:off + n]
        arrays = {"stats_acc": stats,
                  "model": np.asarray(self.eng.model_bytes(), dtype=np.uint8),
                  "host_count": c.count, "host_elevated_sum": c.elevated_sum, "host_x_sum": c.x_sum,
                  "host_xx": c.xx}
        meta = {"model": self.model_name, "seed": self.seed, "learn": self.learn, "windows": self.k,
                "windows_folded_device": int(self.eng.windows_folded) + len(pending),
                "windows_folded_host": self.windows_folded_host, "n_domains": N_DOMAINS}
        return arrays, meta

    def restore(self, arrays: Dict[str, np.ndarray], meta: Dict[str, object]) -> None:
        """Resume from ``state()``: the same model family is required; statistics, the model on
        the device and the fold counters continue where the checkpoint left them."""
        if meta.get("model") != self.model_name or int(meta.get("n_domains", N_DOMAINS)) != N_DOMAINS:
            raise ValueError(f"checkpoint of model {meta.get('model')!r} cannot resume {self.model_name!r}")
        # the learned Bayes is refit on the device from the statistics; other models keep the image
        model = np.zeros(0, np.uint8) if self.device_refit else np.asarray(arrays["model"], dtype=np.uint8)
        self.eng.restore(np.asarray(arrays["stats_acc"], dtype=np.float64), model,
                         int(meta.get("windows_folded_device", 0)))
        self.cum_stats = SufficientStats(count=np.array(arrays["host_count"], dtype=np.float64),
                                         elevated_sum=np.array(arrays["host_elevated_sum"], dtype=np.float64),
                                         x_sum=np.array(arrays["host_x_sum"], dtype=np.float64),
                                         xx=np.array(arrays["host_xx"], dtype=np.float64))
        self.windows_folded_host = int(meta.get("windows_folded_host", 0))
        if not self.device_refit and self.learn and self.cum_stats.count.sum() > 0:
            if self.model_name == "lda" and self.cum_stats.count.sum() > 32:
                self.model = LDA.fit(self.cum_stats)
            else:
                self.model = NaiveBayes.learned(self.cum_stats, **self.learned_kw)

    def save_checkpoint(self, path: str, extra_meta: Optional[Dict[str, object]] = None) -> None:
        from ..utils import checkpoint

        arrays, meta = self.state()
        meta.update(extra_meta or {})
        checkpoint.save(path, arrays, meta)

    def load_checkpoint(self, path: str) -> Dict[str, object]:
        from ..utils import checkpoint

        arrays, meta = checkpoint.load(path)
        self.restore(arrays, meta)
        return meta

    def host_model(self):
        """The model currently on the device, as a host LinearPosteriorModel (reporting)."""
        if not self.device_refit:
            return self.model
        st = self.eng.stats_acc()
        s = SufficientStats(count=st[1024:1024 + N_DOMAINS].copy(),
                            elevated_sum=st[:1024].reshape(32, 32)[:16, :N_DOMAINS].copy(),
                            x_sum=st[:1024].reshape(32, 32)[16:, :N_DOMAINS].copy(),
                            xx=st[:1024].reshape(32, 32)[16:, 16:].copy())
        return NaiveBayes.learned(s, **self.learned_kw)


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
    """Ring window source: the BPF ring buffer (``ring``: a pinned map opened with
    Ringbuf.open_pinned, or an emulated one) plus the optional user-space event and span rings,
    handed to a WindowPipeline as DMA ranges.

    ``cut()`` is the live protocol (the agent is the clock): publish epoch k into mislo_cfg
    (``cfg_set``: the emulated array, or the real map's BpfMap update), then snapshot every
    ring's producer position; records a probe stamps from then on carry the new tag, records
    stamped before it keep theirs and decode against the bases the window ships."""

    def __init__(self, pipe: WindowPipeline, ring=None, user_ring=None, span_ring=None, cfg_set=None,
                 shared: bool = False, flush=None):
        """``shared``: the rings have other consumers too (the node's other GPU workers, agent
        --gpus N): this source never moves a ring's consumer position, it only reports how far
        it is done (``done()``); the agent's controller frees ring space up to the slowest."""
        from ..runtime import load

        self.rt = load()
        self.pipe = pipe
        self.ring, self.user_ring, self.span_ring = ring, user_ring, span_ring
        if cfg_set is None and ring is not None and getattr(ring, "emulated", False):
            cfg_set = lambda i, v: ring.cfg_set(i, v)  # noqa: E731
        self.cfg_set = cfg_set
        self.flush = flush  # the cut's flush of the probes' per-CPU staging batches (BPF rings)
        self.clock = records.EpochClock()
        # page-lock the rings so windows DMA straight from them. Only the first mapping of the
        # double-mapped BPF ring data is registered (page-locking the second copy would count the
        # same pages twice in the agent's RSS): a window that wraps is two DMA segments, placed
        # back to back on the device, so a record split by the wrap is whole again there
        self.direct = {}
        if ring is not None:
            self.direct["ring"] = pipe.eng.register_host(ring.data_address, ring.size)
            self.kpos = ring.consumer_pos
            self.kmask = ring.size - 1
        # user-space producers' records: 64-byte EVENT, 32-byte USER32 or 24-byte USER24, per ring
        self.user_rec = int(user_ring.rec_size) if user_ring is not None else 64
        if self.user_rec not in (16, 24, 32, 64):
            raise ValueError(f"user ring holds {self.user_rec}-byte records (EVENT = 64, USER32 = 32, USER24 = 24, "
                             "USER16 = 16)")
        if user_ring is not None:
            self.direct["user"] = pipe.eng.register_host(user_ring.address, user_ring.capacity * self.user_rec)
            self.upos = user_ring.tail
        if span_ring is not None:
            self.direct["spans"] = pipe.eng.register_host(span_ring.address, span_ring.capacity * 64)
            self.spos = span_ring.tail
        self.shared = shared
        self.kernel_done = self.kpos if ring is not None else 0
        self.kernel_seen = self.kernel_done  # end of the kernel ranges of every reaped window
        self.user_done = self.upos if user_ring is not None else 0
        self.span_done = self.spos if span_ring is not None else 0
        # kernel ranges count batch records (RS ring bytes, BS rows each)
        self.pending: List[tuple] = []   # (k, kernel ranges [(pos, n, window cut)], user n, span n, h2d released)
        self.late: List[tuple] = []      # kernel ranges a window found still being written: (pos, n, window)
        self.late_dropped = 0            # late records too old for the 4 epoch bases of a later window
        self.last: Dict[str, int] = {}
        self.host_s = 0.0
        self.n = 0
        self.resubmitted = 0
        self.carried = 0   # records past a window's budget, summed over windows (should stay 0)
        self.reap_s = self.submit_s = 0.0  # host time: waiting for / reading back finished windows, submitting

    def publish_epoch(self, now_ns: Optional[int] = None) -> int:
        v = self.clock.publish(int(now_ns if now_ns is not None else time.time_ns()))
        if self.cfg_set is not None:
            self.cfg_set(self.rt.CFG_EPOCH, v)
        return v

    def cut(self, now_ns: Optional[int] = None) -> Cut:
        """Close the window at ``now_ns``: new epoch first, then every CPU's staging batches onto
        the ring (``flush``: collector/bpf.py BpfMaps.flush_cpus), then the ring snapshots."""
        t = int(now_ns if now_ns is not None else time.time_ns())
        self.publish_epoch(t)
        if self.flush is not None:
            self.flush()
        return Cut(kernel=self.ring.producer_pos if self.ring is not None else 0,
                   user=self.user_ring.head if self.user_ring is not None else 0,
                   spans=self.span_ring.head if self.span_ring is not None else 0,
                   bases=self.clock.bases(), t_ns=t)

    # ---- ring space --------------------------------------------------------------------------
    def reap(self, keep: Optional[int] = None) -> None:
        """Free ring space of windows whose DMAs (user / span rings) or results (BPF ring) are in;
        with ``keep``, first wait until at most ``keep`` windows are outstanding (a window's
        packet is read before a later window's results overwrite its host buffer)."""
        eng = self.pipe.eng
        while self.pending and (eng.query(self.pending[0][0]) or (keep is not None and len(self.pending) > keep)):
            k, ranges, nu, ns, released = self.pending.pop(0)
            eng.wait(k)
            if not released:
                self._release_user(nu, ns)
            fb = int(eng.packet(k)[sum(PACKET_LAYOUT[:7])])  # ring state: first busy row (-1 = none)
            if fb >= 0:  # batch records from fb's on were still being written: re-submit them
                skip = fb // BS
                for pos, n, k0 in ranges:  # k0: the window whose cut first took the range
                    if skip >= n:
                        skip -= n
                        continue
                    self.late.append((pos + RS * skip, n - skip, k0))
                    self.resubmitted += BS * (n - skip)
                    skip = 0
            if ranges:
                self.kernel_seen = max(self.kernel_seen, max(p + RS * n for p, n, _ in ranges))
        if self.ring is not None:
            # ring space is free up to the decoded records, short of the first range still needed:
            # a late range, or one a window in flight holds (a re-submitted range lies behind
            # ranges already decoded)
            hold = min([p for p, _, _ in self.late] + [p for e in self.pending for p, _, _ in e[1]], default=None)
            self.kernel_done = max(self.kernel_done, min(hold, self.kernel_seen) if hold is not None else self.kernel_seen)
            if not self.shared:
                self.ring.set_consumer_pos(max(self.ring.consumer_pos, self.kernel_done))
        for e in self.pending:  # user / span ring space is free once the DMA that read it is done
            if not e[4] and eng.h2d_done(e[0]):
                self._release_user(e[2], e[3])
                e[4] = True

    def _release_user(self, nu: int, ns: int) -> None:
        self.user_done += nu
        self.span_done += ns
        if self.shared:
            return
        if self.user_ring is not None and nu:
            self.user_ring.release(nu)
        if self.span_ring is not None and ns:
            self.span_ring.release(ns)

    def done(self) -> Tuple[int, int, int]:
        """(BPF ring byte position, user-space records, spans) this source no longer needs."""
        return int(self.kernel_done), int(self.user_done), int(self.span_done)

    def _kernel_segments(self, pos: int, nbytes: int) -> List[Tuple[int, int]]:
        """[(address, bytes)] of BPF ring bytes [pos, pos + nbytes) in the first data mapping."""
        idx = pos & self.kmask
        first = min(nbytes, self.ring.size - idx)
        out = [(self.ring.data_address + idx, first)]
        if nbytes > first:
            out.append((self.ring.data_address, nbytes - first))
        return out

    def _ring_ranges(self, start: int, stop: int, rec: int, base: int, cap_pos: int, max_n: int):
        """[(address, bytes)] of records [start, stop) of a ring of ``cap_pos`` record slots."""
        n = max(0, min(stop - start, max_n))
        out, pos, left = [], start, n
        while left:
            idx = pos & (cap_pos - 1)
            take = min(left, cap_pos - idx)
            out.append((base + idx * rec, take * rec))
            pos += take
            left -= take
        return out, n

    def stage(self, cut: Cut, n_groups: int, labels: Optional[np.ndarray] = None, with_labels: Optional[bool] = None,
              learn: Optional[bool] = None) -> Dict[str, int]:
        """Submit the window up to ``cut``; returns what went in."""
        t0 = time.perf_counter()
        pipe = self.pipe
        self.reap(keep=pipe.nb - 1)
        t1 = time.perf_counter()
        self.reap_s += t1 - t0
        budget = pipe.sig_cap
        k_ranges, kern = [], []
        n_k = 0
        if self.ring is not None:
            late, self.late = self.late, []
            for pos, n, k0 in late:
                # A record of window k0 carries the epoch tag of window k0 or k0 - 1; window
                # pipe.k decodes tags against the bases of windows pipe.k - 3 .. pipe.k, so from
                # pipe.k - k0 = 3 on the tag would name a newer epoch (a timestamp shifted by whole
                # windows): such records are dropped and counted instead.
                if pipe.k - k0 >= 3:
                    self.late_dropped += BS * n
                    continue
                take = min(n, (budget - n_k) // BS)
                if take < n:
                    self.late.append((pos + RS * take, n - take, k0))
                if take:
                    k_ranges.append((pos, take, k0))
                    kern += self._kernel_segments(pos, RS * take)
                    n_k += BS * take
            span_b = cut.kernel - self.kpos
            if span_b % RS:
                raise RuntimeError("BPF ring holds records of another size (the probes emit 8-slot batches only)")
            take = min(span_b // RS, (budget - n_k) // BS)
            self.carried += BS * (span_b // RS - take)
            if take:
                k_ranges.append((self.kpos, take, pipe.k))
                kern += self._kernel_segments(self.kpos, RS * take)
                n_k += BS * take
                self.kpos += RS * take
        user, n_u = [], 0
        if self.user_ring is not None:
            cap = self.user_ring.capacity
            user, n_u = self._ring_ranges(self.upos, cut.user, self.user_rec, self.user_ring.address, cap,
                                          min(pipe.user_cap, budget - n_k))
            self.carried += max(0, cut.user - self.upos) - n_u
            self.upos += n_u
        spans, n_s = [], 0
        if self.span_ring is not None:
            spans, n_s = self._ring_ranges(self.spos, cut.spans, 64, self.span_ring.address, self.span_ring.capacity,
                                           pipe.span_cap)
            self.carried += max(0, cut.spans - self.spos) - n_s
            self.spos += n_s
        wl = labels is not None if with_labels is None else with_labels
        t2 = time.perf_counter()
        k = pipe.submit(kern, user, spans, n_groups, labels, cut.bases, with_labels=wl, learn=learn,
                        user_rec=self.user_rec)
        self.submit_s += time.perf_counter() - t2
        self.pending.append([k, k_ranges, n_u, n_s, False])
        self.host_s += time.perf_counter() - t0
        self.n += 1
        self.last = {"k": k, "n_kernel": n_k, "n_user": n_u, "n_spans": n_s, "n_events": n_k + n_u}
        return self.last

    def step(self, n_groups: int, labels=None, cut: Optional[Cut] = None, with_labels: Optional[bool] = None) -> int:
        """cut (live, unless given) -> submit; returns the window index."""
        c = cut if cut is not None else self.cut()
        return self.stage(c, n_groups, labels, with_labels)["k"]

    def group_sli(self, k: int) -> np.ndarray:
        """[groups, 2] spans and TTFT-SLO breaches per incident group of window k (device-counted)."""
        return self.pipe.results(k, self.pipe.group_cap)["sli"].astype(np.float64)

    def drain(self) -> None:
        self.pipe.drain()
        self.reap(keep=0)


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


def build_replay_images(windows, shift=None, window_ns: int = 1_000_000_000, sim_ring=None,
                        user_rec: int = 64) -> List[ReplayImage]:
    """Run replay windows through the native probe model (one epoch per window cut, published
    at the window start): kernel-signal events become framed batch records of EVENT16 slots, GPU-signal
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
        parts = [sim.encode(np.ascontiguousarray(kev[early]), flush=False)]
        sim_ring.cfg_set(rt.CFG_EPOCH, clock.publish(int(w.t0_ns)))
        # the window ends at the next cut: every CPU's staged batch is flushed into it
        parts.append(sim.encode(np.ascontiguousarray(kev[~early]), flush=True))
        payload = np.concatenate(parts)
        uev = np.ascontiguousarray(w.events[~km])
        out.append(ReplayImage(framed=rt.frame_records(payload), spans=np.ascontiguousarray(w.spans),
                               user=records.to_user(uev, user_rec), bases=clock.bases(),
                               n_groups=w.n_groups,
                               labels=np.asarray(w.group_labels, dtype=np.int32), domains=list(w.group_domains),
                               n_kernel=int(km.sum())))
    return out


def build_shard_images(windows, world: int, pods, window_ns: int = 1_000_000_000,
                       user_rec: int = 64) -> List[List[ReplayImage]]:
    """Split rings: each replay window as the node's producers would have written it into the
    workers' ring sets -- kernel and user-space records by their pod's owner, spans by incident
    group (collector/bpf.py ShardRouter), every ring through its own probe model. Returns, per
    window, one ReplayImage per worker (the same epoch bases in each)."""
    import dataclasses

    from ..collector.bpf import ShardRouter

    router = ShardRouter(world)
    router.set_pods(*pods)
    per_shard = []
    for r in range(world):
        ws = []
        for w in windows:
            ev = w.events[router.pod_shard(w.events["pod_id"]) == r]
            sp = w.spans[router.span_shard(w.spans) == r]
            ws.append(dataclasses.replace(w, events=np.ascontiguousarray(ev), spans=np.ascontiguousarray(sp)))
        per_shard.append(build_replay_images(ws, window_ns=window_ns, user_rec=user_rec))
    return [[per_shard[r][j] for r in range(world)] for j in range(len(windows))]
