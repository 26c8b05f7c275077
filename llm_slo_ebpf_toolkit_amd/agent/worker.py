"""Window workers of the node agent: one per GPU (``agent --gpus N``).

REF runs one agent per node and fans its per-probe readers into one stream
(/root/reference/deploy/k8s/daemonset.yaml:1-20, pkg/collector/ringbuf.go:97-112). On an MI355X
node the agent's window engine can use every GPU of the node, so the agent splits into:

* the **controller** (the agent process, agent/daemon.py): the window clock and the node's only
  ``mislo_cfg`` writer (epochs, node id, emit floors), the cuts of the node's rings, pod
  discovery and the OTLP receiver (the pod -> service table), metrics, outputs, webhook, the
  overhead guard over the whole process tree. It never initialises HIP;
* one **worker per GPU** (a spawned process; ``LocalWorker`` runs the same core in-process when
  the node uses one GPU): a WindowPipeline on its GPU. Worker r owns the services s with
  (s - 1) % N == r, so an incident is scored entirely on one GPU; cross-service trace joins go
  through the engine's trace-row exchange, node-wide histograms through its packet all-reduce,
  and worker 0 receives every worker's incident results through the all-gather (RCCL over xGMI;
  gloo for the CPU engine). Two ways to split the node's stream:

  - **split rings** (``split``, the default with N > 1): every producer writes each record to the
    ring set of the worker owning it (collector/bpf.py ShardRouter: kernel and user-space records
    by their pod's service, spans by incident group; the probes through ``mislo_shards``, the
    rocprofiler tool through the shared pod -> shard table, the OTLP receiver and the procfs
    sampler in the agent). Worker r DMAs and decodes only its own rings -- 1/N of the node's
    bytes -- and frees them itself;
  - **shared rings**: every worker DMAs the whole window and group sharding drops the records of
    services it does not own on the device (decode.hip ``shard_owns``). Workers never move ring
    consumer positions: each reports how far it is done and the controller frees ring space up
    to the slowest worker.

Protocol (multiprocessing pipes, pickled, O(groups) bytes per window): controller -> worker
``("window", cut, n_groups, pods)`` every window, ``("stop",)``; worker -> controller one reply per
window with its release positions, its ring accounting and -- worker 0 only -- the previous
window's node-wide packet and all workers' incident results.

Failure: a worker that dies (or stops answering) breaks the communicator for all of them. The
controller (agent/daemon.py Agent._restart_workers) then stops every worker and starts fresh
processes for the surviving GPUs -- a new communicator (RCCL id / gloo port), world N - 1, the
services re-sharded over them -- which resume from the ring positions already released; the
windows that were in flight are read again (at least once).
"""

from __future__ import annotations

import collections
import os
import time
import traceback
from dataclasses import dataclass, field
from typing import Deque, Dict, List, Optional, Tuple

import numpy as np

RING_TAIL = 8  # ring accounting slots at the packet's tail (pipeline/window.py PACKET_LAYOUT[-1])


@dataclass
class WorkerSpec:
    rank: int
    world: int
    device: int
    engine: str                 # gpu | cpu
    source: str                 # bpf | shm (replay rings are shm rings)
    ring_name: str              # RingNames prefix
    pin_dir: str
    user_rec: int
    sig_cap: int
    span_cap: int
    group_cap: int              # incident groups per worker: ceil(G / world) on every worker (the all-gather
                                # of the results needs equal blocks)
    user_cap: int
    window_ms: float
    ttft_slo_ms: float
    halo_ms: float
    import_cap: int
    xchg_cap: int
    model_image: bytes
    pods: Optional[Tuple[np.ndarray, np.ndarray]] = None
    master: Tuple[str, int] = ("127.0.0.1", 0)   # gloo rendezvous (cpu engine)
    env: Dict[str, str] = field(default_factory=dict)
    halo_windows: int = 3       # earlier windows resident on the device for the halo
    split: bool = False         # split rings: this worker's own ring set (RingNames.of(ring_name, rank))
    app_image: bytes = b""      # the application evidence model (ops/engine.py app_model_bytes); empty: off


def groups_of(rank: int, world: int, n_groups: int) -> int:
    """Incident groups g < n_groups with g % world == rank (local index g // world)."""
    return len(range(rank, n_groups, world))


def merge_results(parts: List[dict], n_groups: int) -> dict:
    """Every worker's local incident results -> the node's, in global group order
    (group g = local g // world of worker g % world)."""
    world = len(parts)
    out = {}
    for key in ("post", "conf", "feat", "pred", "evbits", "sli", "app", "late"):
        if key not in parts[0]:
            continue
        ref = np.asarray(parts[0][key])
        arr = np.zeros((n_groups,) + ref.shape[1:], dtype=ref.dtype)
        for r, p in enumerate(parts):
            n = groups_of(r, world, n_groups)
            arr[r::world][:n] = np.asarray(p[key])[:n]
        out[key] = arr
    return out


class PrevJoiner:
    """The controller's side of the workers' collected windows: each worker reports a window when
    its own chain is done, so one reply may carry none, one or several of them, and the workers
    need not report a window in the same reply. A window is complete once every worker has
    reported it; complete windows come out in window order, each as the workers' parts in rank
    order (rank 0's carries the node-wide packet and every worker's incidents)."""

    def __init__(self, world: int):
        self.world = int(world)
        self.parts: Dict[int, Dict[int, dict]] = {}

    def add(self, replies) -> List[List[dict]]:
        for r in replies:
            for p in r.get("prevs", ()):
                self.parts.setdefault(int(p["k"]), {})[int(r["rank"])] = p
        out = []
        for k in sorted(self.parts):
            if len(self.parts[k]) < self.world:
                break
            got = self.parts.pop(k)
            out.append([got[i] for i in sorted(got)])
        return out

    def reset(self, world: int) -> None:
        self.world = int(world)
        self.parts.clear()


class WorkerCore:
    """One GPU's share of the node's windows (the body of a worker process, or of LocalWorker)."""

    def __init__(self, spec: WorkerSpec, comm=None, group=None, shared: bool = True, rings=None):
        """``rings``: the controller's own ring objects (in-process worker); a worker process maps
        the rings itself (the pinned BPF ring, the named shared-memory rings)."""
        from ..collector import bpf
        from ..pipeline.window import RingWindowSource, WindowPipeline
        from ..runtime import load

        self.spec = spec
        shard = spec.rank if spec.split else 0
        if rings is None:
            rt = load()
            names = bpf.RingNames.of(spec.ring_name, shard)
            if spec.source == "bpf":
                ring = rt.Ringbuf.open_pinned(os.path.join(spec.pin_dir, "mislo_events" + (str(shard) if shard else "")))
            else:
                ring = rt.Ringbuf.attach_shm(names.ring)
            rings = (ring, rt.HostRing(0, spec.user_rec, names.user, True), rt.HostRing(0, 64, names.spans, True))
        ring, user, spans = rings
        self.rings = rings
        self.pipe = WindowPipeline(spec.sig_cap, spec.span_cap, spec.group_cap, spec.device, comm, model="bayes",
                                   learn=False, window_ms=2000.0, user_cap=spec.user_cap,
                                   ttft_slo_ms=spec.ttft_slo_ms, halo_ms=spec.halo_ms, halo_windows=spec.halo_windows,
                                   import_cap=spec.import_cap,
                                   xchg_cap=spec.xchg_cap, shard=(spec.rank, spec.world), engine=spec.engine,
                                   group=group, model_image=np.frombuffer(spec.model_image, dtype=np.uint8),
                                   split_rings=spec.split)
        # the controller publishes the epochs: this source never writes mislo_cfg. Split rings are
        # this worker's alone: it frees their space itself
        self.src = RingWindowSource(self.pipe, ring, user, spans, cfg_set=lambda i, v: None,
                                    shared=shared and not spec.split)
        if spec.pods is not None:
            self.pipe.eng.set_pods(*spec.pods)
        if spec.app_image:
            from ..ops.engine import app_from_bytes

            img = np.frombuffer(spec.app_image, dtype=np.uint8)
            self.pipe.eng.set_app_model(img)
            self.pipe.app = self.pipe.model.app = app_from_bytes(img)
        self.pending: Deque[Tuple[int, float, int]] = collections.deque()
        self.windows = 0
        self.collect_s = self.collect_wait_s = 0.0  # host time collecting finished windows / waiting for them

    @classmethod
    def adopt(cls, spec: WorkerSpec, pipe, src) -> "WorkerCore":
        """A worker core around a pipeline and ring source built elsewhere (bench.py: trained and
        warmed up on the same engine before its timed windows run through this worker path)."""
        core = cls.__new__(cls)
        core.spec, core.pipe, core.src = spec, pipe, src
        core.rings = (src.ring, src.user_ring, src.span_ring)
        core.pending = collections.deque()
        core.windows = 0
        core.collect_s = core.collect_wait_s = 0.0
        return core

    @property
    def max_pending(self) -> int:
        """Windows staged but not yet collected, at most: the engine's buffers minus the one the
        next stage reuses (that window's results must have been read first)."""
        return max(1, int(self.pipe.nb) - 1)

    def window(self, cut, n_groups: int, pods=None, labels=None) -> dict:
        """Stage window k; return, under "prevs", what the controller needs of the earlier windows
        that are finished: every one whose chain is done (at the agent's window period, window
        k-1), and the oldest ones regardless once max_pending are in flight (back-to-back
        windows: the next stage reuses the oldest window's buffer). Collection never waits for a
        window younger than that, so window k+1's copies are issued while windows k-1 and k
        compute (waiting for k-1 here put one window's copy time plus the host's turnaround on
        every window: profiles/r4_timeline/). ``labels``: incident labels for the device's
        confusion matrix (the benchmark's replay windows; the agent has none)."""
        if pods is not None and len(pods[0]):
            self.pipe.eng.set_pods(*pods)
        t0 = time.perf_counter()
        r = self.src.stage(cut, n_groups, labels, with_labels=labels is not None, learn=False)
        host_us = 1e6 * (time.perf_counter() - t0)
        out = {"rank": self.spec.rank, "k": r["k"], "staged": r, "done": self.src.done()}
        self.pending.append((r["k"], host_us, n_groups))
        prevs = []
        while len(self.pending) > 1 and (len(self.pending) > self.max_pending or
                                         self.pipe.eng.query(self.pending[0][0])):
            prevs.append(self._collect(*self.pending.popleft()))
        out["prevs"] = prevs
        self.windows += 1
        return out

    def start_at(self, kernel: int, user: int, spans: int) -> dict:
        """Start reading the rings at these positions (the controller's fresh start: records
        produced while this process spawned are skipped -- older than 3 cuts, their epoch tags
        would decode against the wrong bases -- and the ids they defined were reset). A split
        ring set is this worker's alone: its skipped space is freed here."""
        src = self.src
        if src.ring is not None:
            kernel = max(int(kernel), src.kpos)
            src.kpos = src.kernel_done = src.kernel_seen = kernel
            if not src.shared:
                src.ring.set_consumer_pos(max(src.ring.consumer_pos, kernel))
        if src.user_ring is not None:
            du = max(0, int(user) - src.upos)
            src.upos += du
            src._release_user(du, 0)
        if src.span_ring is not None:
            ds = max(0, int(spans) - src.spos)
            src.spos += ds
            src._release_user(0, ds)
        return {"rank": self.spec.rank, "done": src.done()}

    def collect(self, timeout_s: float) -> dict:
        """Every staged window whose chain finishes within ``timeout_s`` (oldest first), polled --
        the controller's early emission: window k leaves as soon as the device is done with it,
        not at the next cut. A window still computing at the deadline stays pending (the next
        ``window`` or ``collect`` takes it)."""
        deadline = time.perf_counter() + max(0.0, float(timeout_s))
        prevs = []
        while self.pending:
            k = self.pending[0][0]
            while not self.pipe.eng.query(k):
                if time.perf_counter() >= deadline:
                    return {"rank": self.spec.rank, "prevs": prevs}
                time.sleep(2e-4)
            prevs.append(self._collect(*self.pending.popleft()))
        if prevs:  # the collected windows' ring space is free now, not at the next cut: the rings
            self.src.reap()  # need one window of headroom instead of two
        return {"rank": self.spec.rank, "prevs": prevs}

    def _collect(self, k: int, host_us: float, n_groups: int) -> dict:
        pipe = self.pipe
        t0 = time.perf_counter()
        pipe.wait(k)
        t1 = time.perf_counter()
        self.collect_wait_s += t1 - t0
        try:
            return self._read(k, host_us, n_groups)
        finally:
            self.collect_s += time.perf_counter() - t0

    def _read(self, k: int, host_us: float, n_groups: int) -> dict:
        pipe = self.pipe
        pk = np.asarray(pipe.eng.packet(k), dtype=np.float64)
        d = {"k": k, "ring": pk[-RING_TAIL:].copy(), "host_us": host_us, "latency_ms": float(pipe.window_ms(k)[0])}
        if self.spec.rank == 0:  # the node-wide packet and every worker's incidents (all-gathered)
            d["packet"] = pk
            d["results"] = pipe.results_all(k, n_groups) if self.spec.world > 1 else [pipe.results(k, n_groups)]
        return d

    def stop(self) -> dict:
        out = {"rank": self.spec.rank, "done": None, "prevs": []}
        while self.pending:
            out["prevs"].append(self._collect(*self.pending.popleft()))
        self.src.drain()
        out["done"] = self.src.done()
        out["summary"] = self.pipe.summary() if self.spec.rank == 0 else None
        return out

    def close(self) -> None:
        self.pipe.eng.close()


# ---------------------------------------------------------------------------------------
# process plumbing
# ---------------------------------------------------------------------------------------

def worker_main(spec: WorkerSpec, conn) -> None:
    """Spawned worker process: comm bring-up, then one reply per window until "stop"."""
    os.environ.update(spec.env)
    core = None
    group = None
    try:
        comm = None
        if spec.world > 1 and spec.engine == "gpu":
            from ..ops import load_agent

            mod = load_agent()
            if spec.rank == 0:  # the communicator's id travels through the controller
                uid = mod.unique_id()
                conn.send(("uid", uid))
            else:
                uid = conn.recv()[1]
            comm = (uid, spec.rank, spec.world)
        elif spec.world > 1:
            import torch.distributed as dist

            os.environ.update(MASTER_ADDR=spec.master[0], MASTER_PORT=str(spec.master[1]))
            dist.init_process_group("gloo", rank=spec.rank, world_size=spec.world)
            group = dist.group.WORLD
        core = WorkerCore(spec, comm=comm, group=group, shared=True)
        conn.send(("ready", {"rank": spec.rank, "pid": os.getpid(), "device": spec.device}))
        while True:
            msg = conn.recv()
            if msg[0] == "window":
                conn.send(("window", core.window(*msg[1:])))
            elif msg[0] == "collect":
                conn.send(("collect", core.collect(*msg[1:])))
            elif msg[0] == "start_at":
                conn.send(("start_at", core.start_at(*msg[1:])))
            elif msg[0] == "stop":
                conn.send(("stopped", core.stop()))
                break
            else:
                raise ValueError(f"unknown worker message {msg[0]!r}")
    except (EOFError, KeyboardInterrupt):
        pass
    except Exception:  # noqa: BLE001 - reported to the controller, then fatal
        try:
            conn.send(("error", traceback.format_exc()))
        except (OSError, BrokenPipeError):
            pass
        raise
    finally:
        if core is not None:
            core.close()
        if group is not None:
            import torch.distributed as dist

            dist.destroy_process_group()


class WorkerError(RuntimeError):
    def __init__(self, msg: str, rank: Optional[int] = None):
        super().__init__(msg)
        self.rank = rank


class RemoteWorker:
    """Controller-side handle of a spawned worker process."""

    def __init__(self, spec: WorkerSpec, ctx):
        self.spec = spec
        self.conn, child = ctx.Pipe()
        self.proc = ctx.Process(target=worker_main, args=(spec, child), name=f"mislo-worker-{spec.rank}", daemon=True)
        self.proc.start()
        child.close()

    @property
    def pid(self) -> int:
        return int(self.proc.pid or 0)

    def recv(self, timeout: float = 600.0):
        if not self.conn.poll(timeout):
            raise WorkerError(f"worker {self.spec.rank} did not answer in {timeout:.0f} s", self.spec.rank)
        try:
            msg = self.conn.recv()
        except (EOFError, OSError) as exc:
            raise WorkerError(f"worker {self.spec.rank} exited (code {self.proc.exitcode})", self.spec.rank) from exc
        if msg[0] == "error":
            raise WorkerError(f"worker {self.spec.rank} failed:\n{msg[1]}", self.spec.rank)
        return msg

    def ready(self) -> bool:
        return self.conn.poll(0)

    @property
    def alive(self) -> bool:
        return self.proc.is_alive()

    def send(self, msg) -> None:
        self.conn.send(msg)

    def close(self, timeout: float = 30.0) -> None:
        self.proc.join(timeout)
        if self.proc.is_alive():
            self.proc.terminate()
            self.proc.join(10)
        if self.proc.is_alive():
            self.proc.kill()
            self.proc.join(5)


class LocalWorker:
    """The same core in the controller's process (a node agent on one GPU: no extra process)."""

    def __init__(self, spec: WorkerSpec, rings=None):
        self.spec = spec
        self.core = WorkerCore(spec, shared=False, rings=rings)
        self._reply = None

    @property
    def pid(self) -> int:
        return os.getpid()

    def send(self, msg) -> None:
        if msg[0] == "window":
            self._reply = ("window", self.core.window(*msg[1:]))
        elif msg[0] == "collect":
            self._reply = ("collect", self.core.collect(*msg[1:]))
        elif msg[0] == "start_at":
            self._reply = ("start_at", self.core.start_at(*msg[1:]))
        elif msg[0] == "stop":
            self._reply = ("stopped", self.core.stop())

    def recv(self, timeout: float = 600.0):
        r, self._reply = self._reply, None
        return r

    def ready(self) -> bool:
        return True

    alive = True

    def close(self, timeout: float = 30.0) -> None:
        self.core.close()


class WorkerPool:
    """The node's workers: bring-up (RCCL id relay), per-window fan-out / fan-in, and the ring
    space release up to the slowest worker."""

    def __init__(self, specs: List[WorkerSpec], rings, in_process: bool = False):
        import multiprocessing as mp

        self.rings = rings  # the controller's own mappings: (BPF ring, user ring, span ring)
        self.world = len(specs)
        if in_process:
            if self.world != 1:
                raise ValueError("in-process workers: exactly one")
            self.workers = [LocalWorker(specs[0], rings)]
        else:
            ctx = mp.get_context("spawn")
            self.workers = [RemoteWorker(s, ctx) for s in specs]
            try:
                if self.world > 1 and specs[0].engine == "gpu":
                    uid = self.workers[0].recv()[1]
                    for w in self.workers[1:]:
                        w.send(("uid", uid))
                for w in self.workers:
                    w.recv()  # ("ready", info)
            except BaseException:
                self.close()
                raise
        self.in_process = in_process
        self.split = bool(specs[0].split) and self.world > 1
        r = rings
        self._rel_user = r[1].tail if r[1] is not None else 0
        self._rel_spans = r[2].tail if r[2] is not None else 0

    def pids(self) -> List[int]:
        return [w.pid for w in self.workers]

    def window(self, cut, n_groups: int, pods=None, timeout: float = 600.0) -> List[dict]:
        """``cut``: one Cut of the shared rings, or (split rings) a list with each worker's own.
        Raises WorkerError naming the first worker found dead (the others may be blocked in a
        collective with it, so the replies are gathered while watching every process), or the
        first one silent for ``timeout`` s."""
        for w in self.workers:
            c = cut[w.spec.rank] if isinstance(cut, (list, tuple)) and not hasattr(cut, "kernel") else cut
            try:
                w.send(("window", c, groups_of(w.spec.rank, self.world, n_groups), pods))
            except (OSError, BrokenPipeError) as exc:
                raise WorkerError(f"worker {w.spec.rank} is gone ({exc})", w.spec.rank) from exc
        replies = self._gather(timeout)
        self._release(replies)
        return replies

    def collect(self, wait_s: float, timeout: float = 600.0) -> List[dict]:
        """Every worker's windows that finish within ``wait_s`` (WorkerCore.collect): the
        controller emits window k as soon as every worker is done with it."""
        for w in self.workers:
            try:
                w.send(("collect", float(wait_s)))
            except (OSError, BrokenPipeError) as exc:
                raise WorkerError(f"worker {w.spec.rank} is gone ({exc})", w.spec.rank) from exc
        return self._gather(max(timeout, wait_s + 30.0))

    def start_at(self, positions, timeout: float = 120.0) -> List[dict]:
        """Every worker starts reading at ``positions`` -- one (kernel, user, spans) of the shared
        rings, or (split rings) a list with each worker's own -- and the skipped ring space is
        freed."""
        for w in self.workers:
            pos = positions[w.spec.rank] if isinstance(positions, list) else positions
            try:
                w.send(("start_at",) + tuple(int(x) for x in pos))
            except (OSError, BrokenPipeError) as exc:
                raise WorkerError(f"worker {w.spec.rank} is gone ({exc})", w.spec.rank) from exc
        replies = self._gather(timeout)
        self._release(replies)
        return replies

    def _gather(self, timeout: float) -> List[dict]:
        replies: List[Optional[dict]] = [None] * self.world
        deadline = time.monotonic() + timeout
        while any(r is None for r in replies):
            got = False
            for i, w in enumerate(self.workers):
                if replies[i] is None and w.ready():
                    replies[i] = w.recv()[1]
                    got = True
            if got:
                continue
            dead = self.dead_ranks()
            if dead:
                raise WorkerError(f"worker {dead[0]} exited", dead[0])
            if time.monotonic() > deadline:
                late = next(i for i, r in enumerate(replies) if r is None)
                raise WorkerError(f"worker {late} did not answer in {timeout:.0f} s", late)
            time.sleep(0.0005)
        return replies

    def dead_ranks(self) -> List[int]:
        return [w.spec.rank for w in self.workers if not w.alive]

    def _release(self, replies: List[dict]) -> None:
        if self.in_process or self.split:
            return  # the single source / every split-ring worker frees its rings itself
        ring, user, spans = self.rings
        dones = [r["done"] for r in replies if r.get("done") is not None]
        if not dones:
            return
        k = min(d[0] for d in dones)
        if ring is not None and k > ring.consumer_pos:
            ring.set_consumer_pos(k)
        u = min(d[1] for d in dones)
        if user is not None and u > self._rel_user:
            user.release(u - self._rel_user)
            self._rel_user = u
        s = min(d[2] for d in dones)
        if spans is not None and s > self._rel_spans:
            spans.release(s - self._rel_spans)
            self._rel_spans = s

    def stop(self) -> List[dict]:
        for w in self.workers:
            w.send(("stop",))
        replies = []
        for w in self.workers:
            try:
                replies.append(w.recv(120)[1])
            except WorkerError:
                replies.append({"rank": w.spec.rank, "done": None})
        self._release(replies)
        return replies

    def close(self, timeout: float = 30.0) -> None:
        for w in self.workers:
            w.close(timeout)
