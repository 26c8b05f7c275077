"""Multi-GPU node agent on CPU: the benchmark self-launches its ranks, the agent
splits one node's stream over N window workers (group sharding, agent/worker.py) and two
spawned workers running the CPU engine over gloo reproduce the single-process window exactly;
the node id is stable across processes."""

import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_self_launches_its_ranks():
    """`bench.py --gpus 2` with no launcher env starts 2 ranks itself (fresh interpreters, the
    parent never touches the GPU) and rank 0's JSON reports the world the ranks formed."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-probe"],
                         capture_output=True, text=True, env=env, timeout=240, check=True).stdout
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["gpus_requested"] == 2
    assert sorted(r[0] for r in d["ranks"]) == [0, 1] and sorted(r[1] for r in d["ranks"]) == [0, 1]
    assert len({r[2] for r in d["ranks"]}) == 2  # two processes


def test_node_id_is_stable_across_processes():
    code = ("from llm_slo_ebpf_toolkit_amd.collector.bpf import stable_node_id; "
            "print(stable_node_id('mi355x-node-07'))")
    ids = set()
    for seed in ("1", "2", "3"):
        env = dict(os.environ, PYTHONHASHSEED=seed)
        ids.add(subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, cwd=ROOT,
                               check=True).stdout.strip())
    assert len(ids) == 1
    v = int(ids.pop())
    assert 1 <= v <= 0xFFFE


def test_merge_results_places_every_group_once():
    from llm_slo_ebpf_toolkit_amd.agent.worker import groups_of, merge_results

    G, W = 11, 3
    parts = []
    for r in range(W):
        n = groups_of(r, W, G)
        g = np.arange(r, G, W)
        parts.append({"post": np.tile(g[:, None], (1, 16)).astype(float), "conf": g.astype(float),
                      "feat": np.tile(g[:, None], (1, 16)).astype(np.float32), "pred": g.astype(np.int32),
                      "evbits": np.zeros((n, 16), np.uint32), "sli": np.tile(g[:, None], (1, 2)).astype(np.uint32)})
    m = merge_results(parts, G)
    np.testing.assert_array_equal(m["pred"], np.arange(G))
    np.testing.assert_array_equal(m["sli"][:, 0], np.arange(G))


def joiner_windows(replies, world):
    """Every finished window of a run's replies (one list per pool.window / pool.stop call), as
    the workers' parts in rank order (the controller's PrevJoiner)."""
    from llm_slo_ebpf_toolkit_amd.agent.worker import PrevJoiner

    j = PrevJoiner(world)
    out = []
    for rep in replies:
        out.extend(j.add(rep))
    assert not j.parts, "a window some worker never reported"
    return out


def _windows(n_win=3, seed=11):
    from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator
    from llm_slo_ebpf_toolkit_amd.pipeline.window import build_replay_images

    cfg = ReplayConfig(scenario="full", n_nodes=2, pods_per_node=8, n_services=8, events_per_window=3000,
                       spans_per_window=160, seed=seed)
    g = ReplayGenerator(cfg)
    wins = [g.next_window() for _ in range(n_win)]
    sn = (g.pod_svc.astype(np.uint32) << np.uint32(16)) | g.pod_node.astype(np.uint32)
    return wins, build_replay_images(wins, user_rec=24), (g.pod_ids.astype(np.uint32), sn)


def _spec(r, world, tag, pods, port=0, engine="cpu", device=0, halo_ms=2000.0, split=False):
    from llm_slo_ebpf_toolkit_amd.agent.worker import WorkerSpec, groups_of
    from llm_slo_ebpf_toolkit_amd.models.bayes import NaiveBayes
    from llm_slo_ebpf_toolkit_amd.ops.engine import model_bytes

    return WorkerSpec(rank=r, world=world, device=device, engine=engine, source="shm", ring_name=tag, pin_dir="",
                      user_rec=24, sig_cap=8192, span_cap=512, group_cap=groups_of(0, world, 8), user_cap=4096,
                      window_ms=1000.0, ttft_slo_ms=800.0, halo_ms=halo_ms, import_cap=16384,
                      xchg_cap=512 if world > 1 else 0, model_image=model_bytes(NaiveBayes.ref()).tobytes(),
                      pods=pods, master=("127.0.0.1", port), split=split)


def _run_pool(world, imgs, pods, tag, ring_bytes=1 << 22, engine="cpu", late_pods=None, halo_ms=2000.0):
    """``late_pods`` (window index, (pod ids, svc|node)): the pod table arrives at that window's
    cut, as the OTLP receiver's first spans of the pods would deliver it."""
    import socket

    from llm_slo_ebpf_toolkit_amd.agent.worker import WorkerPool, merge_results
    from llm_slo_ebpf_toolkit_amd.collector import bpf
    from llm_slo_ebpf_toolkit_amd.pipeline.window import Cut

    names = bpf.RingNames.of(tag)
    ring, user, spans = bpf.create_rings(names, ring_bytes, 1 << 14, 1 << 12, user_rec=24)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    pool = WorkerPool([_spec(r, world, tag, pods, port, engine, r if engine == "gpu" else 0, halo_ms)
                       for r in range(world)],
                      (ring, user, spans), in_process=world == 1 and engine == "cpu")
    out = []
    try:
        replies = []
        for j, img in enumerate(imgs):
            assert ring.append_framed(img.framed)
            assert user.push(img.user) == len(img.user) and spans.push(img.spans) == len(img.spans)
            upd = late_pods[1] if late_pods is not None and late_pods[0] == j else None
            replies.append(pool.window(Cut(ring.producer_pos, user.head, spans.head, img.bases), 8, upd))
        replies.append(pool.stop())
        for prev in joiner_windows(replies, world):
            out.append({"packet": prev[0]["packet"], "res": merge_results(prev[0]["results"], 8),
                        "events": sum(int(p["ring"][5]) for p in prev)})
        # every worker is done with every record: the controller freed the rings completely
        assert ring.consumer_pos == ring.producer_pos and user.size == 0 and spans.size == 0
    finally:
        pool.close()
    return out


@pytest.mark.timeout(300)
def test_two_cpu_workers_reproduce_the_single_process_window():
    """The same windows through one in-process worker and through two spawned workers (CPU
    engine, gloo): node-wide packet (histograms, status, value sums, join counters: all-reduced),
    every incident's features / posteriors / predictions / SLO counts, and the node's event
    count are identical -- group sharding loses and duplicates nothing, the halo included."""
    wins, imgs, pods = _windows()
    tag = f"/mislo-mg-{os.getpid()}"
    one = _run_pool(1, imgs, pods, tag + "-a")
    two = _run_pool(2, imgs, pods, tag + "-b")
    assert len(one) == len(two) == len(imgs)
    for j, (a, b) in enumerate(zip(one, two)):
        n = 256 + 48 + 18 + 8  # hist, status, misc, dbg
        np.testing.assert_array_equal(a["packet"][:n], b["packet"][:n], err_msg=f"window {j}")
        for key in ("feat", "pred", "sli", "evbits"):
            np.testing.assert_array_equal(a["res"][key], b["res"][key], err_msg=f"window {j} {key}")
        np.testing.assert_allclose(a["res"]["post"], b["res"]["post"], rtol=1e-12, atol=1e-15)
        assert a["events"] == b["events"] > 0
        assert (a["res"]["sli"][:, 0] > 0).all()


@pytest.mark.timeout(300)
def test_pods_learned_after_their_contexts_were_defined_shard_like_one_process():
    """on a bpf source the pod -> service table fills only once the OTLP
    receiver sees a pod's spans, after the kernel defined the pod's contexts. Sharding must use
    the service the pod table holds when a record is decoded, not the one stored with its context
    at definition time (svc 0, which kept every such record on GPU 0 and left the other GPUs'
    services without them). Pods arrive at window 1's cut; from then on two workers equal one."""
    wins, imgs, pods = _windows(n_win=4)
    tag = f"/mislo-late-{os.getpid()}"
    one = _run_pool(1, imgs, None, tag + "-a", late_pods=(1, pods), halo_ms=0.0)
    two = _run_pool(2, imgs, None, tag + "-b", late_pods=(1, pods), halo_ms=0.0)
    for j in range(1, len(imgs)):
        a, b = one[j], two[j]
        for key in ("feat", "pred", "sli"):
            np.testing.assert_array_equal(a["res"][key], b["res"][key], err_msg=f"window {j} {key}")
        assert a["events"] == b["events"] > 0


def _run_split(world, shard_imgs, pods, tag, ring_bytes=1 << 22, engine="cpu"):
    """``agent --gpus N`` on split rings: worker r's own ring set holds only the records and
    spans of the services it owns (what the node's producers write through ShardRouter)."""
    import socket

    from llm_slo_ebpf_toolkit_amd.agent.worker import WorkerPool, merge_results
    from llm_slo_ebpf_toolkit_amd.collector import bpf
    from llm_slo_ebpf_toolkit_amd.pipeline.window import Cut

    sets = bpf.create_shard_rings(tag, world, ring_bytes, 1 << 14, 1 << 12, user_rec=24)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    pool = WorkerPool([_spec(r, world, tag, pods, port, engine, r if engine == "gpu" else 0, split=True)
                       for r in range(world)], sets[0])
    out, direct = [], []
    try:
        replies = []
        for imgs in shard_imgs:
            cuts = []
            for (ring, user, spans), img in zip(sets, imgs):
                assert ring.append_framed(img.framed)
                assert user.push(img.user) == len(img.user) and spans.push(img.spans) == len(img.spans)
                cuts.append(Cut(ring.producer_pos, user.head, spans.head, img.bases))
            direct.append([len(img.framed) + img.user.nbytes for img in imgs])
            replies.append(pool.window(cuts, 8))
        replies.append(pool.stop())
        for prev in joiner_windows(replies, world):
            out.append({"packet": prev[0]["packet"], "res": merge_results(prev[0]["results"], 8),
                        "events": sum(int(p["ring"][5]) for p in prev)})
        # every worker freed its own rings completely (nobody else consumes them)
        for ring, user, spans in sets:
            assert ring.consumer_pos == ring.producer_pos and user.size == 0 and spans.size == 0
    finally:
        pool.close()
    return out, direct


@pytest.mark.timeout(300)
def test_two_workers_on_split_rings_reproduce_the_single_process_window():
    """the node's stream split at the source. Each of two workers DMAs and
    decodes only its own ring set (half of the window's bytes), and the node-wide packet, every
    incident's results and the node's event count equal one process reading one ring."""
    from llm_slo_ebpf_toolkit_amd.pipeline.window import build_shard_images

    wins, imgs, pods = _windows()
    tag = f"/mislo-split-{os.getpid()}"
    one = _run_pool(1, imgs, pods, tag + "-a")
    two, direct = _run_split(2, build_shard_images(wins, 2, pods, user_rec=24), pods, tag + "-b")
    assert len(one) == len(two) == len(imgs)
    for j, (a, b) in enumerate(zip(one, two)):
        n = 256 + 48 + 18 + 8  # hist, status, misc, dbg
        np.testing.assert_array_equal(a["packet"][:n], b["packet"][:n], err_msg=f"window {j}")
        for key in ("feat", "pred", "sli", "evbits"):
            np.testing.assert_array_equal(a["res"][key], b["res"][key], err_msg=f"window {j} {key}")
        np.testing.assert_allclose(a["res"]["post"], b["res"]["post"], rtol=1e-12, atol=1e-15)
        assert a["events"] == b["events"] > 0
    whole = [len(i.framed) + i.user.nbytes for i in imgs]
    for j, per in enumerate(direct):  # each worker's share of the bytes is about half
        assert sum(per) >= whole[j] and all(0.3 * whole[j] < x < 0.7 * whole[j] for x in per), (per, whole[j])


def _net_packet(p, n):
    """The packet's first n elements with the low-confidence count net of the tier-4 overlap: the
    GPU probe reports (raw low, overlap) in dbg[1:3], the CPU engine the net count and 0."""
    q = np.array(p[:n], dtype=np.float64)
    lo = 256 + 48 + 18 + 1  # dbg[1]
    q[lo] -= q[lo + 1]
    q[lo + 1] = 0.0
    return q


def _assert_same_windows(ref, got):
    assert len(ref) == len(got)
    for j, (a, b) in enumerate(zip(ref, got)):
        n = 256 + 48 + 18 + 8  # hist, status, misc, dbg
        pa, pb = _net_packet(a["packet"], n), _net_packet(b["packet"], n)
        bad = np.nonzero(pa != pb)[0]
        assert not len(bad), f"window {j}: packet elements {bad.tolist()} differ: {pa[bad].tolist()} vs {pb[bad].tolist()}"
        for key in ("feat", "pred", "sli", "evbits"):
            np.testing.assert_array_equal(a["res"][key], b["res"][key], err_msg=f"window {j} {key}")
        np.testing.assert_allclose(a["res"]["post"], b["res"]["post"], rtol=1e-9, atol=1e-12)
        assert a["events"] == b["events"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_gpu_worker_reproduces_the_cpu_oracle():
    """The agent's spawned GPU window worker (the shipped WindowEngine on the BPF-layout rings)
    against the single-process CPU engine on the same windows, halo included."""
    wins, imgs, pods = _windows()
    tag = f"/mislo-mg1-{os.getpid()}"
    _assert_same_windows(_run_pool(1, imgs, pods, tag + "-c"), _run_pool(1, imgs, pods, tag + "-g", engine="gpu"))


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_gpu_worker_with_late_pods_reproduces_the_cpu_oracle():
    """Pods learned after their contexts were defined: the device decode resolves a record's
    service through the pod table at decode time (decode.hip), as the oracle does -- the
    service + node tier joins those records from the window the pods arrive in."""
    wins, imgs, pods = _windows(n_win=4)
    tag = f"/mislo-mgl-{os.getpid()}"
    _assert_same_windows(_run_pool(1, imgs, None, tag + "-c", late_pods=(1, pods)),
                         _run_pool(1, imgs, None, tag + "-g", engine="gpu", late_pods=(1, pods)))


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_two_gpu_workers_over_rccl_reproduce_the_cpu_oracle():
    """Two GPU window workers (one per GPU, joined by the engine's RCCL communicator: packet
    all-reduce, incident all-gather, in-window trace-row all-gather) against the single-process
    CPU engine on the same windows: node-wide packet and every incident identical, posteriors to
    f64 rounding. Needs two GPUs: RCCL refuses two ranks on one device."""
    import torch

    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs (RCCL refuses two ranks on one device)")
    wins, imgs, pods = _windows()
    tag = f"/mislo-mg-{os.getpid()}"
    _assert_same_windows(_run_pool(1, imgs, pods, tag + "-c"), _run_pool(2, imgs, pods, tag + "-g", engine="gpu"))


@pytest.mark.timeout(300)
def test_agent_cpu_engine_with_two_workers_end_to_end(tmp_path):
    """`agent --engine cpu --gpus 2 --source replay`: the controller spawns two workers, emits
    schema-valid attributions for the node's incidents, and checkpoints / resumes its state."""
    code = f"""
import io, json, os, sys
sys.path.insert(0, {ROOT!r})
from llm_slo_ebpf_toolkit_amd.agent.daemon import Agent, AgentOptions
from llm_slo_ebpf_toolkit_amd.contracts import validator
if __name__ == "__main__":
    out = io.StringIO()
    o = AgentOptions(engine="cpu", source="replay", gpus=2, window_events=4096, window_spans=256, window_groups=8,
                     window_ms=400, count=5, metrics_bind="", output="stdout", ring_name="/mislo-e2e-%d" % os.getpid(),
                     config="", min_confidence=0.0, state_dir={str(tmp_path)!r})
    a = Agent(o, out_stream=out)
    rc = a.run_windows(max_windows=5)
    recs = [json.loads(x) for x in out.getvalue().splitlines()]
    schema = validator.compiled("incident-attribution")
    assert all(schema.is_valid(r) for r in recs), recs[:1]
    print(json.dumps({{"rc": rc, "n": len(recs), "services": sorted({{r["service"] for r in recs}}),
                      "windows": a.windows_done, "workers": len(a.pool.workers)}}))
    a.close()
"""
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=280, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["rc"] == 0 and d["workers"] == 2 and d["windows"] == 5
    assert d["n"] > 0 and len(d["services"]) >= 4
    st = [f for f in os.listdir(tmp_path) if f.endswith(".state.json")]
    assert st, os.listdir(tmp_path)
    with open(tmp_path / st[0]) as fh:
        state = json.load(fh)
    assert state["windows"] == 5 and state["burn"]["hist"]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("split", [False, True])
def test_agent_survives_a_worker_killed_mid_run(tmp_path, split):
    """`agent --engine cpu --gpus 3 --source replay`: one of the three worker processes is
    SIGKILLed after a few windows. The controller notices (the survivors may be blocked in a
    collective with it), stops them, starts fresh workers for the 2 surviving GPUs with a new
    communicator, and keeps emitting schema-valid attributions for every service."""
    code = f"""
import io, json, os, signal, sys, threading, time
import numpy as np
sys.path.insert(0, {ROOT!r})
from llm_slo_ebpf_toolkit_amd.agent.daemon import Agent, AgentOptions
from llm_slo_ebpf_toolkit_amd.contracts import validator
if __name__ == "__main__":
    out = io.StringIO()
    o = AgentOptions(engine="cpu", source="replay", gpus=3, window_events=4096, window_spans=256, window_groups=8,
                     window_ms=400, metrics_bind="", output="stdout", ring_name="/mislo-kill-%d" % os.getpid(),
                     config="", min_confidence=0.0, split_rings={split!r})
    a = Agent(o, out_stream=out)
    killed = {{}}

    def killer():
        while a.windows_done < 3:
            time.sleep(0.05)
        victim = a.pool.workers[1].pid
        killed["pid"], killed["at"] = victim, a.windows_done
        os.kill(victim, signal.SIGKILL)

    threading.Thread(target=killer, daemon=True).start()
    # kernel-ring records (context ids the fresh workers must learn again): per window, the incident
    # groups whose features hold a DNS value (a kernel-ring signal resolved to its pod's service)
    kern = []
    orig = a._attributions

    def spy(G, names, res, t_ns, model):
        kern.append((a.metrics.worker_restarts.value(), int(np.isfinite(res["feat"][:, 0]).sum())))
        return orig(G, names, res, t_ns, model)

    a._attributions = spy
    rc = a.run_windows(max_windows=10)
    recs = [json.loads(x) for x in out.getvalue().splitlines()]
    schema = validator.compiled("incident-attribution")
    assert all(schema.is_valid(r) for r in recs), recs[:1]
    after = [r for r in recs if int(r["incident_id"].split("-")[1]) > 0]
    print(json.dumps({{"rc": rc, "n": len(recs), "services": sorted({{r["service"] for r in recs}}),
                      "windows": a.windows_done, "workers": len(a.pool.workers), "killed": killed,
                      "restarts": a.metrics.worker_restarts.value(), "gauge": a.metrics.workers.value(),
                      "kern": kern}}))
    a.close()
"""
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=280, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["killed"] and d["killed"]["at"] >= 3
    assert d["rc"] == 0 and d["restarts"] == 1 and d["workers"] == 2 and d["gauge"] == 2
    assert d["windows"] == 10 and d["n"] > 0 and len(d["services"]) >= 4
    assert "restarting on 2 worker(s)" in p.stderr
    # after the restart the ids are defined again, so kernel-ring records keep resolving
    # to their pods' services (not context 0): past the restart's transition (the producers switch
    # over at their next window) every window joins DNS records to groups
    after = [n for r, n in d["kern"] if r >= 1]
    assert len(after) >= 4 and min(after[2:]) > 0, d["kern"]


def test_windows_that_wrap_the_bpf_ring_equal_unwrapped_windows():
    """Only the first mapping of the double-mapped BPF ring is page-locked: a window that wraps
    goes as two DMA segments placed back to back, records split by the wrap included, and the
    results equal those of the same windows in a ring that never wraps."""
    wins, imgs, pods = _windows(n_win=5)
    tag = f"/mislo-wr-{os.getpid()}"
    big = _run_pool(1, imgs, pods, tag + "-a")
    small = _run_pool(1, imgs, pods, tag + "-b", ring_bytes=1 << 18)  # a later window wraps
    assert sum(im.framed.size for im in imgs) > (1 << 18)
    for j, (a, b) in enumerate(zip(big, small)):
        np.testing.assert_array_equal(a["packet"], b["packet"], err_msg=f"window {j}")
        for key in ("feat", "pred", "sli", "evbits"):
            np.testing.assert_array_equal(a["res"][key], b["res"][key], err_msg=f"window {j} {key}")


@pytest.mark.timeout(600)
def test_bench_runs_the_agents_worker_path_on_two_ranks(tmp_path):
    """`bench.py --gpus 2` (self-launched ranks, the host oracle engine over
    gloo) times the agent's topology: each rank is a window worker on its own split ring set
    (agent/worker.py WorkerCore.window per step) and rank 0 runs the controller's per-window
    epilogue (Agent._emit_window) over every timed window, measured on its own."""
    out = tmp_path / "bench.json"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--engine", "cpu", "--model", "bayes",
                        "--events", "4096", "--spans", "256", "--services", "8", "--windows", "2", "--heldout", "3",
                        "--paced-windows", "0", "--steps", "3", "--warmup", "1", "--ring-mib", "16",
                        "--train-windows", "0", "--out", str(out)],
                       capture_output=True, text=True, timeout=580, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads(out.read_text())
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["value"] > 0
    assert "split rings" in d["topology"] and "WorkerCore.window" in d["topology"]
    # every node-wide incident of the timed windows was scored; those with SLO impact (the replay's
    # faulted groups breach the TTFT SLO) became attributions on the controller
    assert d["incidents_scored_timed_windows"] == 3 * 2 * 8
    assert 0 < d["attributions_emitted_timed"] <= d["incidents_scored_timed_windows"]
    assert d["host_epilogue_us_per_window"] > 0


def test_bench_trains_the_learned_model_on_the_host_engine(tmp_path):
    """`bench.py --engine cpu` with the learned model: the host engine accumulates the labelled
    windows' sufficient statistics as the device does (its packets' statistics block), so the
    model trained from random-init priors scores the timed windows (it scored none before)."""
    out = tmp_path / "bench.json"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--engine", "cpu", "--events", "16384",
                        "--spans", "1024", "--services", "16", "--windows", "2", "--heldout", "0",
                        "--paced-windows", "0", "--steps", "3", "--warmup", "1", "--ring-mib", "16",
                        "--train-windows", "8", "--train-events", "16384", "--train-spans", "1024", "--out", str(out)],
                       capture_output=True, text=True, timeout=580, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads(out.read_text())
    assert d["training"]["windows"] == 8 and d["training"]["incidents_trained"] > 0
    assert d["macro_f1_timed_windows"] >= 0.9
    assert d["incidents_scored_timed_windows"] == 3 * 16
    assert 0 < d["attributions_emitted_timed"] <= d["incidents_scored_timed_windows"]


def test_prev_joiner_emits_windows_once_every_worker_reported_them():
    """Workers report a window when their own chain is done (agent/worker.py WorkerCore.window):
    worker 1 may still be computing window 3 when worker 0 reports it. The controller emits a
    window once both reported it, in window order, with rank 0's part first."""
    from llm_slo_ebpf_toolkit_amd.agent.worker import PrevJoiner

    j = PrevJoiner(2)
    p = lambda r, k: {"k": k, "rank_tag": r}  # noqa: E731
    assert j.add([{"rank": 1, "prevs": [p(1, 3)]}, {"rank": 0, "prevs": []}]) == []
    out = j.add([{"rank": 0, "prevs": [p(0, 3), p(0, 4)]}, {"rank": 1, "prevs": []}])
    assert [[x["rank_tag"] for x in w] for w in out] == [[0, 1]] and out[0][0]["k"] == 3
    out = j.add([{"rank": 1, "prevs": [p(1, 4), p(1, 5)]}, {"rank": 0, "prevs": [p(0, 5)]}])
    assert [w[0]["k"] for w in out] == [4, 5] and not j.parts
    j.add([{"rank": 0, "prevs": [p(0, 6)]}])
    j.reset(1)  # a worker was lost: the pool restarts with one worker and re-reads those windows
    assert j.add([{"rank": 0, "prevs": [p(0, 6)]}])[0][0]["k"] == 6
