"""The agent's side of the probes' maps, and the producers that stand in for the kernel.

REF designs a kernel -> user path (pkg/collector/ringbuf.go:56-150, probe_manager.go:25-185)
that no binary constructs. NEW's agent opens the maps the loader pinned (``make ebpf-gen`` +
``bpftool prog loadall ... pinmaps /sys/fs/bpf/mislo``; probes/ebpf/Makefile) with raw bpf(2):

* ``mislo_events`` -- the BPF ring buffer the window source consumes (runtime/csrc/bpfring.h);
* ``mislo_cfg``   -- the agent writes the realtime-monotonic clock offset, the node id, the
  per-signal emit floors (the overhead guard raises them to the evidence thresholds before it detaches
  probes: safety.ShedLadder) and the
  epoch it publishes at every window cut;
* ``mislo_pods``  -- cgroup id -> pod id, filled from the node's cgroup tree (pods discovered
  the way REF's ProcMetadataEnricher derives them, pkg/signals/metadata.go:95-118);
* ``mislo_ctxs`` / ``mislo_traces`` -- the kernel's interning maps. The agent never reads them
  per window: every new id reaches it as a definition record ahead of its first use in the
  ring (mislo_probe.h MISLO_INTERN_DEF). It resets them when the context id space runs low.

``EmulatedMaps`` gives the same interface over the emulated ring (tests, CI, the benchmark,
``--source shm``); ``ReplayProducer`` is a separate process that writes seeded fault-replay
windows into emulated rings exactly as the probes and the rocprofiler tool would.
"""

from __future__ import annotations

import os
import struct
import time
from dataclasses import dataclass
from typing import Dict, Iterable, Optional, Tuple

import numpy as np

from . import records

CFG_CLOCK, CFG_NODE, CFG_EPOCH, CFG_TRACE_NEXT, CFG_CTX_NEXT = 0, 1, 124, 125, 126
# replay producer control (emulated maps only; no probe reads it): (generation << 8) | ring sets in
# use. A new generation after a worker restart makes the producer re-route over the surviving
# workers' ring sets and re-intern every id, so the fresh workers see every definition again.
CFG_REPLAY_CTL = 127
PIN_DIR = "/sys/fs/bpf/mislo"


def stable_node_id(name: str) -> int:
    """The node's 16-bit id in [1, 0xFFFE] (mislo_cfg[1], the svc|node join key): the first two
    bytes of the BLAKE2b digest of the node name -- the same in every process and across
    restarts (Python's str hash is salted per process)."""
    import hashlib

    v = int.from_bytes(hashlib.blake2b(str(name).encode("utf-8"), digest_size=2).digest(), "little")
    return min(max(v, 1), 0xFFFE)


def cfg_floor(signal_type: int) -> int:
    return 2 + int(signal_type)


def clock_offset_ns() -> int:
    """CLOCK_REALTIME - CLOCK_MONOTONIC: what the probes add to bpf_ktime_get_ns()."""
    return time.clock_gettime_ns(time.CLOCK_REALTIME) - time.clock_gettime_ns(time.CLOCK_MONOTONIC)


class MapSet:
    """Common agent-side operations over the probes' maps."""

    ring = None

    def cfg_set(self, idx: int, value: int) -> None:  # pragma: no cover - interface
        raise NotImplementedError

    def cfg_get(self, idx: int) -> int:  # pragma: no cover - interface
        raise NotImplementedError

    def set_pod(self, cgroup_id: int, pod_id: int) -> None:  # pragma: no cover - interface
        raise NotImplementedError

    def init(self, node_id: int) -> None:
        self.cfg_set(CFG_CLOCK, clock_offset_ns() & 0xFFFFFFFFFFFFFFFF)
        self.cfg_set(CFG_NODE, int(node_id) & 0xFFFF)

    def set_floor(self, signal_type: int, raw_value: int) -> None:
        self.cfg_set(cfg_floor(signal_type), int(raw_value))

    def ctx_ids_used(self) -> int:
        return int(self.cfg_get(CFG_CTX_NEXT))

    def flush_cpus(self) -> int:
        """The window cut's flush of every CPU's staging batches (after the new epoch is
        published, before the ring positions are read); CPUs flushed. The emulated rings'
        producers flush their own batches."""
        return 0


class EmulatedMaps(MapSet):
    """mislo_cfg lives in the emulated ring's meta page (every shard ring's, with split rings:
    each ring's producers read the epoch and floors from their own ring); pods in a dict."""

    def __init__(self, ring, shard_rings=()):
        self.ring = ring
        self.rings = [ring] + [r for r in shard_rings if r is not None and r is not ring]
        self.pods: Dict[int, int] = {}

    def cfg_set(self, idx: int, value: int) -> None:
        for r in self.rings:
            r.cfg_set(int(idx), int(value) & 0xFFFFFFFFFFFFFFFF)

    def cfg_get(self, idx: int) -> int:
        return int(self.ring.cfg_get(int(idx)))

    def set_pod(self, cgroup_id: int, pod_id: int) -> None:
        self.pods[int(cgroup_id)] = int(pod_id)

    def reset_definitions(self, world: int) -> None:
        """After a worker restart: the replay producer re-routes over ``world`` ring sets and
        re-interns every context / trace id (its next records carry the definitions again)."""
        gen = (self.cfg_get(CFG_REPLAY_CTL) >> 8) + 1
        self.cfg_set(CFG_REPLAY_CTL, (gen << 8) | (int(world) & 0xFF))


class BpfMaps(MapSet):
    """The maps the loader pinned under ``pin_dir`` (needs CAP_BPF / root)."""

    def __init__(self, pin_dir: str = PIN_DIR):
        from ..runtime import load

        rt = load()
        self.pin_dir = pin_dir
        self.ring = rt.Ringbuf.open_pinned(os.path.join(pin_dir, "mislo_events"))
        self.cfg = rt.BpfMap(os.path.join(pin_dir, "mislo_cfg"))
        self.pods = rt.BpfMap(os.path.join(pin_dir, "mislo_pods"))
        self._ctxs = os.path.join(pin_dir, "mislo_ctxs")
        self._traces = os.path.join(pin_dir, "mislo_traces")
        # probes/ebpf/mislo_flush.bpf.c, pinned by the loader (no attachment): run on each CPU at
        # every cut. Without it a quiet CPU's partial batch waits for that CPU's next event.
        self.flush_fd = rt.bpf_obj_get(os.path.join(pin_dir, "progs", "mislo_flush", "mislo_flush"))
        self.cpus = list(range(os.cpu_count() or 1))
        self.flush_errors = 0

    def flush_cpus(self) -> int:
        if self.flush_fd < 0:
            return 0
        from ..runtime import load

        rt = load()
        n = 0
        for c in self.cpus:
            r = rt.bpf_prog_run_on_cpu(self.flush_fd, c)
            if r >= 0:
                n += 1
            elif r != -6:  # -ENXIO: an offline CPU
                self.flush_errors += 1
        return n

    def cfg_set(self, idx: int, value: int) -> None:
        self.cfg.update(struct.pack("<I", int(idx)), struct.pack("<Q", int(value) & 0xFFFFFFFFFFFFFFFF))

    def cfg_get(self, idx: int) -> int:
        v = self.cfg.lookup(struct.pack("<I", int(idx)))
        return 0 if v is None else struct.unpack("<Q", v)[0]

    def set_pod(self, cgroup_id: int, pod_id: int) -> None:
        self.pods.update(struct.pack("<Q", int(cgroup_id)), struct.pack("<I", int(pod_id)))

    def set_shards(self, pod_ids, shards) -> None:
        """mislo_shards: the ring a pod's records go to (split rings, agent --gpus N)."""
        if getattr(self, "_shards", None) is None:
            from ..runtime import load

            try:
                self._shards = load().BpfMap(os.path.join(self.pin_dir, "mislo_shards"))
            except (OSError, RuntimeError):
                self._shards = False
        if not self._shards:
            return
        for p, s in zip(np.asarray(pod_ids).tolist(), np.asarray(shards).tolist()):
            self._shards.update(struct.pack("<I", int(p)), struct.pack("<I", int(s)))

    def reset_definitions(self, world: int) -> None:
        """After a worker restart the fresh workers' context and trace tables are empty, and the
        probes define an id only when they first intern it: clear both interning maps and their
        counters, so every id is defined again -- on every ring that carries it -- by the next
        records (kernel records would otherwise resolve to context 0, no pod)."""
        from ..runtime import load

        self.reset_ctx_ids()
        m = load().BpfMap(self._traces)
        keys, _ = m.items()
        ks = m.info()["key_size"]
        for i in range(0, len(keys), ks):
            m.delete(keys[i:i + ks])
        self.cfg_set(CFG_TRACE_NEXT, 0)

    def reset_ctx_ids(self) -> int:
        """Clear mislo_ctxs and restart its id counter (the agent does this at a window cut when
        the kernel's 2^23 context ids run low; rows are redefined as contexts reappear)."""
        from ..runtime import load

        m = load().BpfMap(self._ctxs)
        keys, _ = m.items()
        ks = m.info()["key_size"]
        n = 0
        for i in range(0, len(keys), ks):
            n += bool(m.delete(keys[i:i + ks]))
        self.cfg_set(CFG_CTX_NEXT, 0)
        return n


def discover_pods(cgroup_root: str = "/sys/fs/cgroup", interner=None) -> Dict[int, Tuple[int, str]]:
    """cgroup id (the directory inode bpf_get_current_cgroup_id() returns on cgroup v2) -> (pod
    id, pod uid) for every kubepods cgroup on the node; pod ids come from ``interner`` (a
    signals.metadata.Interner over pod uids) so they stay stable across scans."""
    from ..signals.metadata import Interner

    interner = interner if interner is not None else Interner()
    out: Dict[int, Tuple[int, str]] = {}
    for dirpath, _dirs, _files in os.walk(cgroup_root):
        base = os.path.basename(dirpath)
        if "pod" not in base:
            continue
        uid = _pod_uid(base)
        if not uid:
            continue
        try:
            ino = os.stat(dirpath).st_ino
        except OSError:
            continue
        out[ino] = (interner.id(uid), uid)
    return out


def _pod_uid(name: str) -> str:
    """kubepods-burstable-pod<uid with _>.slice | pod<uid> -> uid (REF metadata.go:95-118)."""
    i = name.rfind("pod")  # the last one: "kubepods-...-pod<uid>" holds two
    if i < 0:
        return ""
    s = name[i + 3:]
    for suffix in (".slice", ".scope"):
        if s.endswith(suffix):
            s = s[: -len(suffix)]
    s = s.replace("_", "-")
    return s if len(s) >= 32 and all(c in "0123456789abcdef-" for c in s.lower()) else ""


# ---------------------------------------------------------------------------------------
# replay producer (stands in for the kernel probes + the rocprofiler tool + instrumented services)
# ---------------------------------------------------------------------------------------

@dataclass
class RingNames:
    ring: str
    user: str
    spans: str

    @staticmethod
    def of(prefix: str, shard: int = 0) -> "RingNames":
        """The ring set of one worker (``shard`` > 0: agent --gpus N with split rings, worker
        ``shard``'s own kernel / user-space / span rings)."""
        sfx = str(int(shard)) if shard else ""
        return RingNames(prefix + "-bpf" + sfx, prefix + "-events" + sfx, prefix + "-spans" + sfx)

    @staticmethod
    def shard_table(prefix: str) -> str:
        """Shared-memory pod id -> shard byte table the user-space producers route by."""
        return prefix + "-shards"


def shard_of_pod(svcnode: np.ndarray, world: int) -> np.ndarray:
    """The worker that owns a pod's records: its service's (decode.hip shard_owns: service
    s >= 1 -> (s - 1) % world; no service yet -> 0)."""
    svc = (np.asarray(svcnode, dtype=np.uint32) >> np.uint32(16)).astype(np.int64)
    return np.where(svc > 0, (svc - 1) % max(1, world), 0).astype(np.int64)


class ShardRouter:
    """Split rings (agent --gpus N): one ring set per worker, every record written to the ring of
    the worker that owns it -- kernel and user-space records by their pod's service (the pod
    table), spans by their incident group (group g -> worker g % N). Each worker then DMAs and
    decodes only its own share of the node's stream."""

    def __init__(self, world: int, table=None):
        self.world = max(1, int(world))
        self.svc: Dict[int, int] = {}  # pod id -> svc|node
        self.table = table              # shared-memory pod -> shard bytes (numpy view), for the GPU tool

    def set_pods(self, pods: np.ndarray, sn: np.ndarray) -> None:
        sh = shard_of_pod(sn, self.world)
        for p, v, s in zip(np.asarray(pods).tolist(), np.asarray(sn).tolist(), sh.tolist()):
            self.svc[int(p)] = int(v)
            if self.table is not None and 0 <= int(p) < len(self.table):
                self.table[int(p)] = int(s)

    def pod_shard(self, pod_ids: np.ndarray) -> np.ndarray:
        sn = np.array([self.svc.get(int(p), 0) for p in np.asarray(pod_ids).tolist()], dtype=np.uint32)
        return shard_of_pod(sn, self.world)

    def resize(self, world: int) -> Tuple[np.ndarray, np.ndarray]:
        """Re-shard every known pod over ``world`` workers (a worker was lost): the shared table
        follows at once; returns (pods, shards) for the probes' mislo_shards map."""
        self.world = max(1, int(world))
        pods = np.array(sorted(self.svc), dtype=np.int64)
        sh = self.pod_shard(pods) if len(pods) else np.zeros(0, np.int64)
        if self.table is not None:
            for p, s in zip(pods.tolist(), sh.tolist()):
                if 0 <= p < len(self.table):
                    self.table[p] = int(s)
        return pods, sh

    def span_shard(self, spans: np.ndarray) -> np.ndarray:
        return (spans["group_id"].astype(np.int64) % self.world).astype(np.int64)

    def split(self, recs: np.ndarray, shard: np.ndarray):
        """[(shard, records of that shard)] in shard order (stable within a shard)."""
        return [(r, recs[shard == r]) for r in range(self.world)]


def create_shard_rings(prefix: str, world: int, ring_bytes: int, user_records: int, span_records: int,
                       user_rec: int = 16):
    """One ring set per worker (split rings), each sized for its share of the node's stream."""
    return [create_rings(RingNames.of(prefix, r), ring_bytes, user_records, span_records, user_rec)
            for r in range(max(1, int(world)))]


def create_rings(names: RingNames, ring_bytes: int, user_records: int, span_records: int, user_rec: int = 16):
    """Create the emulated BPF ring and the two user-space rings (the agent owns them). The
    user-space ring holds ``user_rec``-byte records: 16 = USER16 slots (what the rocprofiler tool
    and the samplers write into such a ring: a quarter of the PCIe bytes of a 64-byte EVENT, a
    traced record two slots), 24 = USER24, 32 = USER32."""
    from ..runtime import load

    rt = load()
    pow2 = lambda n: 1 << max(12, int(np.ceil(np.log2(max(1, n)))))  # noqa: E731
    return (rt.Ringbuf.create_shm(names.ring, pow2(ring_bytes)),
            rt.HostRing(pow2(user_records), int(user_rec), names.user),
            rt.HostRing(pow2(span_records), 64, names.spans))


def replay_producer_main(names: RingNames, cfg_kwargs: dict, rate_eps: float, window_ms: int, max_windows: int,
                         n_images: int, ready=None, shard_names=None) -> None:
    """Process body: generates ``n_images`` replay windows, then writes one window per
    ``window_ms`` at ``rate_eps``: the kernel-signal records through the probe model (using
    the epoch the agent published, read from the emulated mislo_cfg at write time), the GPU-
    signal records and the spans into the user-space rings. Stops after ``max_windows`` (0 =
    forever). Never touches the GPU. ``shard_names``: the workers' ring sets (split rings): every
    record goes to the ring set of the worker owning its service (ShardRouter), through that
    ring's own probe model (each kernel ring carries its own id definitions)."""
    from ..pipeline.replay import ReplayConfig, ReplayGenerator
    from ..pipeline.window import kernel_event_mask
    from ..runtime import load

    rt = load()
    sets = list(shard_names) if shard_names else [names]
    world = len(sets)
    rbs = [rt.Ringbuf.attach_shm(n.ring) for n in sets]
    users = [rt.HostRing(0, 64, n.user, True) for n in sets]
    spanss = [rt.HostRing(0, 64, n.spans, True) for n in sets]
    # the cycled images keep one fault assignment (window k's halo joins window k+1)
    cfg = ReplayConfig(window_ms=window_ms, fault_hold=max(1, n_images), **cfg_kwargs)
    gen = ReplayGenerator(cfg)
    wins = [gen.next_window() for _ in range(max(1, n_images))]
    sims = [rt.ProbeSim(rb, records.milli_shift_table()) for rb in rbs]
    router = ShardRouter(world)
    router.set_pods(*pod_metadata(cfg_kwargs))
    parts = []
    for w in wins:
        km = kernel_event_mask(w.events)
        kev, uev, sp = w.events[km], w.events[~km], w.spans
        ks, us, ss = router.pod_shard(kev["pod_id"]), router.pod_shard(uev["pod_id"]), router.span_shard(sp)
        parts.append([(np.ascontiguousarray(kev[ks == r]), np.ascontiguousarray(uev[us == r]),
                       np.ascontiguousarray(sp[ss == r])) for r in range(world)])
    if ready is not None:
        ready.send(True)
    period = window_ms / 1000.0
    # the replay's timestamps are re-based onto wall-clock time, one window per period
    t_start = time.time_ns()
    nxt = time.perf_counter()
    j = 0
    ctl = int(rbs[0].cfg_get(CFG_REPLAY_CTL))
    while not max_windows or j < max_windows:
        c = int(rbs[0].cfg_get(CFG_REPLAY_CTL))
        if c != ctl:  # a worker restart: fresh id interning, the surviving workers' ring sets
            ctl = c
            world = max(1, min(len(sets), c & 0xFF))
            sims = [rt.ProbeSim(rb, records.milli_shift_table()) for rb in rbs[:world]]
            router = ShardRouter(world)
            router.set_pods(*pod_metadata(cfg_kwargs))
            parts = []
            for w in wins:
                km = kernel_event_mask(w.events)
                kev, uev, sp = w.events[km], w.events[~km], w.spans
                ks, us, ss = router.pod_shard(kev["pod_id"]), router.pod_shard(uev["pod_id"]), router.span_shard(sp)
                parts.append([(np.ascontiguousarray(kev[ks == r]), np.ascontiguousarray(uev[us == r]),
                               np.ascontiguousarray(sp[ss == r])) for r in range(world)])
        shift = t_start + j * int(period * 1e9) - int(wins[j % len(wins)].t0_ns)
        shard_parts = []
        for r, (kev, uev, sp) in enumerate(parts[j % len(parts)]):
            kev, uev, sp = kev.copy(), uev.copy(), sp.copy()
            for a in (kev, uev, sp):
                nz = a["ts_ns"] != 0
                a["ts_ns"][nz] += shift
            # what the rocprof tool writes into this ring
            shard_parts.append((kev, records.to_user(uev, int(users[r].rec_size)), sp))
        # pace: the window's records go out in 10 slices across its period
        n_sl = 10
        for s in range(n_sl):
            for r, (kev, uev, sp) in enumerate(shard_parts):
                lo_k, hi_k = len(kev) * s // n_sl, len(kev) * (s + 1) // n_sl
                # staged per CPU as the probes do (a batch goes out when full, with a
                # definition, or at the first record after the agent's next epoch)
                sims[r].submit(kev[lo_k:hi_k], flush=False)
                lo_u, hi_u = len(uev) * s // n_sl, len(uev) * (s + 1) // n_sl
                if hi_u > lo_u:
                    users[r].push(uev[lo_u:hi_u])
                lo_s, hi_s = len(sp) * s // n_sl, len(sp) * (s + 1) // n_sl
                if hi_s > lo_s:
                    spanss[r].push(sp[lo_s:hi_s])
            nxt += period / n_sl
            time.sleep(max(0.0, nxt - time.perf_counter()))
        for sim in sims:  # what the agent's cut flush does to a quiet CPU's batch
            sim.flush()
        j += 1


def pod_metadata(cfg_kwargs: dict) -> Tuple[np.ndarray, np.ndarray]:
    """pod id -> svc<<16|node of the replay world (what kubelet metadata gives a live agent)."""
    from ..pipeline.replay import ReplayConfig, ReplayGenerator

    g = ReplayGenerator(ReplayConfig(**cfg_kwargs))
    sn = (g.pod_svc.astype(np.uint32) << np.uint32(16)) | g.pod_node.astype(np.uint32)
    return g.pod_ids.astype(np.uint32), sn


def start_replay_producer(names: RingNames, cfg_kwargs: dict, rate_eps: float, window_ms: int,
                          max_windows: int = 0, n_images: int = 2, shard_names=None):
    """Fork the replay producer (before this process touches the GPU) and wait until it has
    generated its windows."""
    import multiprocessing as mp

    ctx = mp.get_context("fork")
    a, b = ctx.Pipe()
    p = ctx.Process(target=replay_producer_main,
                    args=(names, cfg_kwargs, rate_eps, window_ms, max_windows, n_images, b, shard_names), daemon=True)
    p.start()
    if not a.poll(600):
        raise RuntimeError("replay producer did not start")
    a.recv()
    return p


def iter_chunks(a: np.ndarray, n: int) -> Iterable[np.ndarray]:
    for i in range(0, len(a), n):
        yield a[i:i + n]
