"""First-token SLI records (collector/records.py SPAN_FIRST_TOKEN / SPAN_NO_SLI): a service exports a
request's TTFT when its first token is out (demo/rag_service.py chat.first_token,
llm.slo.ttft_early) and the request span at the end; the receiver (collector/otlp.py) flags the
pair so the request counts once -- the first-token record carries the SLI, the request span does
not count again. Both join: the first-token record brings the request's kernel evidence into the
window its SLI is counted in (a CPU-starved service exports its request spans a window or more
later), the request span adds the pod+conn tier. On both engines the SLI, late and retrieval
counts of a window with the pairs equal those with the request spans alone; the GPU engine's
paired windows equal the host engine's (k_decode_spans / pipeline/cpu.py)."""

import os

import numpy as np
import pytest

from llm_slo_ebpf_toolkit_amd.collector import otlp
from llm_slo_ebpf_toolkit_amd.collector import records as R
from llm_slo_ebpf_toolkit_amd.signals.metadata import Interner

RES = {"service.name": "rag-service", "k8s.pod.uid": "0f1e2d3c-4b5a-6978-8796-a5b4c3d2e1f0", "process.pid": 4242}
T0 = 1_700_000_000_000_000_000


def _json(spans):
    import json

    def av(v):
        if isinstance(v, bool):
            return {"boolValue": v}
        if isinstance(v, float):
            return {"doubleValue": v}
        return {"intValue": str(v)} if isinstance(v, int) else {"stringValue": v}

    return json.dumps({"resourceSpans": [{
        "resource": {"attributes": [{"key": k, "value": av(v)} for k, v in RES.items()]},
        "scopeSpans": [{"scope": {"name": "s"}, "spans": [
            {"traceId": t, "spanId": s, **({"parentSpanId": p} if p else {}), "name": "x", "kind": 2,
             "startTimeUnixNano": str(t0), "endTimeUnixNano": str(t1),
             "attributes": [{"key": k, "value": av(v)} for k, v in a.items()]}
            for t, s, p, t0, t1, a in spans]}]}]}).encode()


def _early(tid, ttft):
    return (tid, "00000000000000f1", "00000000000000a1", T0, T0 + int(ttft * 1e6),
            {"llm.slo.ttft_ms": ttft, "llm.slo.ttft_early": True})


def _final(tid, ttft, retr=None):
    out = [(tid, "00000000000000a1", "", T0, T0 + 900_000_000, {"llm.slo.ttft_ms": ttft, "client.port": 51000,
                                                                  "server.port": 443})]
    if retr is not None:
        out.insert(0, (tid, "00000000000000b1", "00000000000000a1", T0, T0 + 20_000_000,
                       {"llm.slo.retrieval.vectordb_ms": retr}))
    return out


def test_receiver_counts_a_request_once_whichever_record_comes_first():
    m = otlp.SpanMapper(otlp.GroupTable(4), Interner().id)
    a, b, c = (f"{i:032x}" for i in (1, 2, 3))
    # a: first token, then the request span (with its retrieval breakdown)
    r1 = m.records(otlp.parse_json(_json([_early(a, 90.0)])))
    assert len(r1) == 1 and int(r1["flags"][0]) == R.SPAN_FIRST_TOKEN and float(r1["retr_ms"][0]) == 0.0
    r2 = m.records(otlp.parse_json(_json(_final(a, 91.0, retr=150.0))))
    assert len(r2) == 1 and int(r2["flags"][0]) == R.SPAN_NO_SLI
    assert r2["retr_ms"][0] == np.float32(150.0)  # the retrieval folds into the request span, not the early one
    # a2: the retrieval span sent before (or with) the first-token record: the breakdown rides on it
    a2 = f"{5:032x}"
    ret = _final(a2, 0.0, retr=120.0)[0]
    r5 = m.records(otlp.parse_json(_json([ret])))
    assert len(r5) == 0  # a child span: no record, its breakdown waits for the trace's first record
    r6 = m.records(otlp.parse_json(_json([_early(a2, 95.0)])))
    assert r6["retr_ms"][0] == np.float32(120.0)
    r7 = m.records(otlp.parse_json(_json(_final(a2, 96.0))))
    assert int(r7["flags"][0]) == R.SPAN_NO_SLI and float(r7["retr_ms"][0]) == 0.0  # counted once
    # b: the request span alone (a service without first-token export)
    r3 = m.records(otlp.parse_json(_json(_final(b, 50.0))))
    assert int(r3["flags"][0]) == 0
    # c: the request span first, the first-token record after it: the late one is dropped
    m.records(otlp.parse_json(_json(_final(c, 40.0))))
    assert len(m.records(otlp.parse_json(_json([_early(c, 40.0)])))) == 0 and m.early_dropped == 1
    # late flag combines: a first-token record whose deadline passed before the last cut
    m.slo_ms, m.late_before_ns = 10.0, T0 + 50_000_000
    r4 = m.records(otlp.parse_json(_json([_early(f"{4:032x}", 80.0)])))
    assert int(r4["flags"][0]) == R.SPAN_FIRST_TOKEN | R.SPAN_LATE
    # the tables are bounded
    m2 = otlp.SpanMapper(otlp.GroupTable(4), Interner().id)
    m2.retrieval_cap = 3
    for i in range(8):
        m2.records(otlp.parse_json(_json([_early(f"{i + 100:032x}", 5.0)] + _final(f"{i + 200:032x}", 5.0))))
    assert len(m2._early) == 3 and len(m2._final) == 3


def test_rag_service_exports_the_first_token_record():
    from llm_slo_ebpf_toolkit_amd.demo.rag_service import RagService, StubBackend
    from llm_slo_ebpf_toolkit_amd.runtime import load

    rt = load()
    ring = rt.HostRing(64, 64)
    m = otlp.SpanMapper(otlp.GroupTable(4), Interner().id)
    rx = otlp.OtlpSpanReceiver("127.0.0.1:0", m, ring.push).start()
    try:
        svc = RagService(StubBackend(), otlp_endpoint=rx.endpoint, resource={"k8s.pod.uid": RES["k8s.pod.uid"]})
        outs = [svc.chat({"prompt": f"first token {i}", "profile": "chat_short", "max_tokens": 3}) for i in range(3)]
        svc.spans.flush()
    finally:
        rx.stop()
    buf = ring.records_view()[: ring.size * 64].view(R.SPAN)
    assert ring.size == 6
    for o in outs:
        mine = buf[buf["trace_h"] == np.uint64(otlp.trace_hash(o["trace_id"]))]
        assert sorted(int(f) for f in mine["flags"]) == [R.SPAN_NO_SLI, R.SPAN_FIRST_TOKEN]
        early = mine[mine["flags"] == R.SPAN_FIRST_TOKEN][0]
        assert abs(float(early["ttft_ms"]) - o["ttft_ms"]) < 2.0  # the request span's definition, known earlier
        final = mine[mine["flags"] == R.SPAN_NO_SLI][0]
        assert early["conn_h"] == final["conn_h"]  # the request's connection: both join the pod+conn tier
        # the retrieval span leaves when it ends: its breakdown rides on the first-token record, once
        assert float(early["retr_ms"]) > 0 and float(final["retr_ms"]) == 0.0


def _with_first_token(sp, every=2):
    """Every ``every``-th request also as a first-token record (same TTFT), the request flagged."""
    sp = sp.copy()
    idx = np.arange(0, len(sp), every)
    early = sp[idx].copy()
    early["flags"] = R.SPAN_FIRST_TOKEN
    early["retr_ms"] = 0.0
    early["conn_h"] = 0
    sp["flags"][idx] |= R.SPAN_NO_SLI
    out = np.concatenate([early, sp])
    return out[np.argsort(out["ts_ns"], kind="stable")]


def _run(engine, wins, tag, pair):
    from llm_slo_ebpf_toolkit_amd.models.bayes import NaiveBayes
    from llm_slo_ebpf_toolkit_amd.pipeline.window import RingWindowSource, WindowPipeline, build_replay_images
    from tests.test_native_engine import feed, pod_meta, rings

    for w in wins:
        w.spans = _with_first_token(w.spans0) if pair else w.spans0
    imgs = build_replay_images(wins, user_rec=24)
    pipe = WindowPipeline(16384, 1024, 8, model="bayes_gpu", learn=False, user_cap=4096, engine=engine)
    pipe.set_model(NaiveBayes.gpu())
    rb, user, spans = rings(f"ft{tag}", 24)
    src = RingWindowSource(pipe, rb, user, spans)
    pipe.eng.set_pods(*pod_meta(wins[0].gen))
    out = []
    for w, img in zip(wins, imgs):
        k = src.stage(feed(img, rb, user, spans), w.n_groups, img.labels)["k"]
        pk = pipe.packet(k)
        res = {key: np.array(v, copy=True) for key, v in pipe.results(k, w.n_groups).items()}
        out.append((np.array(pk["dbg"][:5], copy=True), np.array(pk["hist"], copy=True), res))
    src.drain()
    pipe.eng.close()
    return out


@pytest.mark.parametrize("engine", ["cpu", pytest.param("gpu", marks=pytest.mark.gpu)])
def test_first_token_records_count_once_and_join(engine):
    from tests.test_native_engine import windows

    wins, gen = windows(n_win=2, seed=7)
    for w in wins:
        w.spans0, w.gen = w.spans.copy(), gen
    plain = _run(engine, wins, f"{engine}{os.getpid()}p", False)
    paired = _run(engine, wins, f"{engine}{os.getpid()}q", True)
    for j, ((d0, h0, r0), (d1, h1, r1)) in enumerate(zip(plain, paired)):
        np.testing.assert_array_equal(h0, h1, err_msg=f"window {j} hist")  # the signals are the same
        for key in ("sli", "late", "app"):  # each request counted once, retrieval on the request span
            np.testing.assert_array_equal(r0[key], r1[key], err_msg=f"window {j} {key}")
        assert r0["sli"][:, 0].sum() == len(wins[j].spans0)
        assert d1[0] > d0[0], f"window {j}: the first-token records join (pairs {d0[0]} -> {d1[0]})"
    if engine == "gpu":  # the paired windows on the device equal the host engine's
        host = _run("cpu", wins, f"h{os.getpid()}q", True)
        for j, ((d1, h1, r1), (dh, hh, rh)) in enumerate(zip(paired, host)):
            # dbg: candidates, low-confidence (the device reports raw and overlap in [1:3], the host
            # the net count and 0), fan-out drops, enriched spans
            net = lambda d: [int(d[0]), int(d[1] - d[2]), int(d[3]), int(d[4])]  # noqa: E731
            assert net(d1) == net(dh), (j, d1, dh)
            np.testing.assert_array_equal(h1, hh, err_msg=f"window {j} hist")
            for key in ("sli", "late", "app", "feat", "pred", "evbits"):
                np.testing.assert_array_equal(r1[key], rh[key], err_msg=f"window {j} {key}")
            np.testing.assert_allclose(r1["post"], rh["post"], rtol=1e-9, atol=1e-12)
