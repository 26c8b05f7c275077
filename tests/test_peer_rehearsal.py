"""Eight GPUs' trace-row exchange rehearsed on one: worker ``me`` of an
8-GPU node runs its own shard of the node's windows (split rings, group sharding) while the seven
other workers' exchange blocks -- each the oracle's selection of that worker's warn-level
trace-tagged rows (oracle.trace_rows -> exchange_blocks) -- are injected where the RCCL
all-gather would deliver them. The native engine's window (features, candidates, per-incident
results, packet) equals the host engine's (pipeline/cpu.py CpuRingEngine, the same contract on
the numpy oracle) with the same blocks; an import capacity below the peers' rows counts the
overflow (dbg[6]) on both engines instead of losing it silently."""

import os

import numpy as np
import pytest

from llm_slo_ebpf_toolkit_amd.collector import bpf
from llm_slo_ebpf_toolkit_amd.pipeline import oracle
from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator

WORLD, XCAP = 8, 1024


def node_windows(n_win=3, seed=17):
    cfg = ReplayConfig(scenario="full", n_nodes=4, pods_per_node=16, n_services=16, events_per_window=32000,
                       spans_per_window=1600, seed=seed)
    g = ReplayGenerator(cfg)
    wins = [g.next_window() for _ in range(n_win)]
    sn = (g.pod_svc.astype(np.uint32) << np.uint32(16)) | g.pod_node.astype(np.uint32)
    return wins, (g.pod_ids.astype(np.uint32), sn)


def peer_blocks(shard_imgs, pods, me):
    """Every worker's exchange block of one window (the oracle's selection of its own rows)."""
    pod_sn = dict(zip(pods[0].tolist(), pods[1].tolist()))
    parts = []
    for r, img in enumerate(shard_imgs):
        table, tmap = oracle.CtxTable(), oracle.TraceMap()
        oracle.apply_ring_defs(img.framed, table, tmap, pod_sn)
        d = oracle.decode_window(img.framed, img.user, table, tmap, img.bases, pod_sn=pod_sn)
        parts.append(oracle.trace_rows(d, len(d.ts)) if r != me else oracle.empty_rows())
    return oracle.exchange_blocks(parts, XCAP), sum(min(len(p.ts), XCAP) for p in parts)


def run(engine, imgs, blocks, pods, me, icap, tag):
    from llm_slo_ebpf_toolkit_amd.models.bayes import NaiveBayes
    from llm_slo_ebpf_toolkit_amd.pipeline.window import Cut, RingWindowSource, WindowPipeline

    names = bpf.RingNames.of(tag)
    ring, user, spans = bpf.create_rings(names, 1 << 22, 1 << 15, 1 << 12, user_rec=64)
    pipe = WindowPipeline(32768, 1024, 2, model="bayes", learn=False, user_cap=8192, halo_ms=2000.0,
                          import_cap=icap, xchg_cap=XCAP, shard=(me, WORLD), split_rings=True, engine=engine)
    pipe.set_model(NaiveBayes.ref())
    pipe.eng.set_pods(*pods)
    src = RingWindowSource(pipe, ring, user, spans)
    out = []
    for img, blk in zip(imgs, blocks):
        pipe.inject_remote(blk, world=WORLD, me=me)
        assert ring.append_framed(img.framed)
        assert user.push(img.user) == len(img.user) and spans.push(img.spans) == len(img.spans)
        # this worker's incident groups: g % 8 == me of the node's 16 (agent/worker.py groups_of)
        k = src.stage(Cut(ring.producer_pos, user.head, spans.head, img.bases), 2, None)["k"]
        pk = pipe.packet(k)
        out.append((pk, {key: np.array(v, copy=True) for key, v in pipe.results(k, 2).items()}))
    src.drain()
    pipe.eng.close()
    return out


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("icap", [7 * XCAP, 600])
def test_seven_peers_blocks_join_like_the_host_engine(icap):
    wins, pods = node_windows()
    from llm_slo_ebpf_toolkit_amd.pipeline.window import build_shard_images

    shards = build_shard_images(wins, WORLD, pods)
    me = 3
    blocks, n_peer = zip(*(peer_blocks(s, pods, me) for s in shards))
    imgs = [s[me] for s in shards]
    assert min(n_peer) > icap or icap > max(n_peer)  # the case this parameter means
    tag = f"/mislo-peer-{os.getpid()}-{icap}"
    gpu = run("gpu", imgs, blocks, pods, me, icap, tag + "-g")
    cpu = run("cpu", imgs, blocks, pods, me, icap, tag + "-c")
    for j, ((pg, rg), (pc, rc)) in enumerate(zip(gpu, cpu)):
        for key in ("hist", "status", "confusion"):
            np.testing.assert_array_equal(pg[key], pc[key], err_msg=f"window {j} {key}")
        # (dbg[5], this worker's own selection beyond XCAP, exists on the device only: the host
        # engine without a group selects nothing)
        np.testing.assert_array_equal(pg["dbg"][[0, 3, 4, 6]], pc["dbg"][[0, 3, 4, 6]], err_msg=f"window {j}")
        for key in ("feat", "pred", "sli", "evbits"):
            np.testing.assert_array_equal(rg[key], rc[key], err_msg=f"window {j} {key}")
        np.testing.assert_allclose(rg["post"], rc["post"], rtol=1e-9, atol=1e-12)
        assert int(pg["dbg"][6]) == max(0, n_peer[j] - icap), (j, pg["dbg"][:8], n_peer[j])
    assert sum(int(p["dbg"][0]) for p, _ in gpu) > 0
