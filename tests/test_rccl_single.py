"""The window engine's RCCL path on a one-GPU box: a one-rank communicator.

RCCL refuses two ranks on one device, so the two-rank tests (test_rccl_pair.py,
test_multigpu_agent.py) skip on the one-GPU box. A communicator of world 1 still runs every
collective the multi-GPU chain issues (engine.hip: the trace-row all-gather between the window's
two halves -- on the compute stream over a split communicator, or on the comm stream --, the packet all-reduce and the incident all-gather on the comm stream, the results
copied from the all-gathered block, the totals accumulated behind the collectives), so the same
windows through an engine with and without one must agree bit for bit: packets, incident
results, features, posteriors and totals. SURVEY §2.4 RCCL table; REF has no collective
(its fan-in is /root/reference/pkg/collector/ringbuf.go:97-112)."""

import numpy as np
import pytest

from test_native_engine import feed, pod_meta, rings, windows

pytestmark = pytest.mark.gpu


def _run(tag, comm, wins, imgs, gen):
    from llm_slo_ebpf_toolkit_amd.pipeline.window import RingWindowSource, WindowPipeline

    pipe = WindowPipeline(16384, 512, 8, comm=comm, model="bayes", learn=False, user_cap=4096, halo_ms=2000.0,
                          import_cap=4096, xchg_cap=1024)
    rb, user, spans = rings(tag)
    src = RingWindowSource(pipe, rb, user, spans)
    pipe.eng.set_pods(*pod_meta(gen))
    out, sent = [], []
    for w, img in zip(wins, imgs):
        k = src.stage(feed(img, rb, user, spans), w.n_groups, img.labels)["k"]
        pk = {key: np.array(v, copy=True) if not isinstance(v, dict) else dict(v) for key, v in pipe.packet(k).items()}
        res = {key: v.copy() for key, v in pipe.results(k, w.n_groups).items()}
        allr = [{key: v.copy() for key, v in r.items()} for r in pipe.results_all(k, w.n_groups)]
        out.append((pk, res, allr))
        sent.append(bytes(pipe.eng.sent_block()) if comm is not None else b"")
    src.drain()
    info = {"has_comm": bool(pipe.eng.has_comm) if hasattr(pipe.eng, "has_comm") else comm is not None,
            "world": int(pipe.eng.world), "totals": np.asarray(pipe.eng.totals(), dtype=np.float64).copy(),
            "sent": sent}
    pipe.eng.close()
    return out, info


@pytest.mark.timeout(120)
@pytest.mark.parametrize("xchg_stream", ["compute", "comm"])
def test_one_rank_rccl_communicator_matches_the_communicator_free_engine(xchg_stream, monkeypatch):
    """xchg_stream: the trace-row exchange on the comm stream with the window's other collectives
    (the default: one communicator, one stream), or on the compute stream over a communicator of
    its own (MISLO_XCHG_STREAM=compute: a split decided on rank 0 and broadcast)."""
    from llm_slo_ebpf_toolkit_amd.ops import load_agent
    from llm_slo_ebpf_toolkit_amd.pipeline.window import build_replay_images

    if xchg_stream == "compute":
        monkeypatch.setenv("MISLO_XCHG_STREAM", "compute")
    else:
        monkeypatch.delenv("MISLO_XCHG_STREAM", raising=False)
    wins, gen = windows(n_win=4, seed=71)
    imgs = build_replay_images(wins)
    solo, solo_info = _run("solo", None, wins, imgs, gen)
    rccl, rccl_info = _run("rccl1", (load_agent().unique_id(), 0, 1), wins, imgs, gen)
    assert rccl_info["world"] == 1
    for j, ((pa, ra, aa), (pb, rb, ab)) in enumerate(zip(solo, rccl)):
        for key in pa:
            if isinstance(pa[key], dict):
                assert pa[key] == pb[key], (j, key)
            else:
                np.testing.assert_array_equal(pa[key], pb[key], err_msg=f"window {j} packet {key}")
        for key in ("feat", "pred", "evbits", "sli", "conf"):
            np.testing.assert_array_equal(ra[key], rb[key], err_msg=f"window {j} results {key}")
        np.testing.assert_allclose(ra["post"], rb["post"], rtol=1e-12, atol=0, err_msg=f"window {j} posteriors")
        # the node-wide incident list of a one-rank node is this GPU's, from the all-gathered block
        assert len(ab) == 1 and len(aa) == 1
        for key in ("feat", "pred", "post", "evbits", "sli"):
            np.testing.assert_array_equal(ab[0][key], rb[key], err_msg=f"window {j} all-gathered {key}")
    assert any(int(r[0]["dbg"][0]) > 0 for r in rccl), "no join candidates: the comparison would be vacuous"
    np.testing.assert_array_equal(solo_info["totals"], rccl_info["totals"])


@pytest.mark.timeout(120)
def test_the_exchange_block_is_the_oracles_trace_row_selection():
    """What this GPU hands the all-gather each window (k_sel_count / k_sel_scan / k_sel_scatter:
    its warn-level trace-tagged local rows, identity dropped, in row order, capped at xchg_cap)
    is byte for byte the oracle's block (oracle.trace_rows -> oracle.exchange_blocks). With one
    rank nothing is imported, so the comparison above never looks at these bytes."""
    from llm_slo_ebpf_toolkit_amd.ops import load_agent
    from llm_slo_ebpf_toolkit_amd.pipeline import oracle
    from llm_slo_ebpf_toolkit_amd.pipeline.window import build_replay_images

    from test_native_engine import pod_meta as _pm

    wins, gen = windows(n_win=4, seed=73)
    imgs = build_replay_images(wins)
    out, info = _run("sel", (load_agent().unique_id(), 0, 1), wins, imgs, gen)
    pods, sn = _pm(gen)
    pod_sn = dict(zip(pods.tolist(), sn.tolist()))
    table, tmap = oracle.CtxTable(), oracle.TraceMap()
    n_sel = []
    for j, (img, blk) in enumerate(zip(imgs, info["sent"])):
        oracle.apply_ring_defs(img.framed, table, tmap, pod_sn)
        d_loc = oracle.decode_window(img.framed, img.user, table, tmap, img.bases)
        mine = oracle.trace_rows(d_loc, len(d_loc.ts))
        ref = oracle.exchange_blocks([mine], 1024)
        got = np.frombuffer(blk, dtype=np.uint8)
        assert got.size == ref.size, (j, got.size, ref.size)
        n_dev = int(got[:4].view(np.uint32)[0])
        assert n_dev == min(len(mine.ts), 1024), (j, n_dev, len(mine.ts))
        w = oracle.XREC.itemsize
        np.testing.assert_array_equal(got[w:w * (1 + n_dev)], ref[w:w * (1 + n_dev)], err_msg=f"window {j}")
        n_sel.append(n_dev)
        # rows beyond the exchange capacity are counted (dbg[5]), never silently lost
        assert int(out[j][0]["dbg"][5]) == max(0, len(mine.ts) - 1024), (j, out[j][0]["dbg"][:8])
    assert min(n_sel) > 0, "no trace rows selected: the comparison would be vacuous"
