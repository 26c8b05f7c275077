"""OTLP/HTTP span receiver (collector/otlp.py): OTLP/JSON and OTLP/proto export requests
become SPAN records on the agent's ids in the span ring; the demo RAG service's exporter
feeds it end to end (REF demo/rag-service/main.go:408-441 -> REF ebpfcorrelator)."""

import json
import struct
import urllib.request

import numpy as np

from llm_slo_ebpf_toolkit_amd.collector import otlp, records
from llm_slo_ebpf_toolkit_amd.signals.metadata import Interner

TID = "4bf92f3577b34da6a3ce929d0e0e4736"


# ---- a minimal OTLP/proto encoder (test side only) -------------------------------------
def _v(n):
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        out.append(b | (0x80 if n else 0))
        if not n:
            return bytes(out)


def _ld(fn, payload):
    return _v(fn << 3 | 2) + _v(len(payload)) + payload


def _fx64(fn, x):
    return _v(fn << 3 | 1) + struct.pack("<Q", x)


def _kv(k, val):
    if isinstance(val, str):
        av = _ld(1, val.encode())
    elif isinstance(val, float):
        av = _fx64(4, struct.unpack("<Q", struct.pack("<d", val))[0])
    else:
        av = _v(3 << 3 | 0) + _v(val & (2**64 - 1))
    return _ld(1, k.encode()) + _ld(2, av)


def _span_pb(trace, span, parent, t0, t1, attrs):
    b = _ld(1, bytes.fromhex(trace)) + _ld(2, bytes.fromhex(span))
    if parent:
        b += _ld(4, bytes.fromhex(parent))
    b += _ld(5, b"chat.request") + _v(6 << 3) + _v(2) + _fx64(7, t0) + _fx64(8, t1)
    for k, v in attrs.items():
        b += _ld(9, _kv(k, v))
    return b


def _request_pb(resource, spans):
    res = b"".join(_ld(1, _kv(k, v)) for k, v in resource.items())
    ss = _ld(1, _ld(1, b"scope")) + b"".join(_ld(2, s) for s in spans)
    return _ld(1, _ld(1, res) + _ld(2, ss))


def _request_json(resource, spans):
    def av(v):
        if isinstance(v, str):
            return {"stringValue": v}
        if isinstance(v, float):
            return {"doubleValue": v}
        return {"intValue": str(v)}

    return json.dumps({"resourceSpans": [{
        "resource": {"attributes": [{"key": k, "value": av(v)} for k, v in resource.items()]},
        "scopeSpans": [{"scope": {"name": "s"}, "spans": [
            {"traceId": t, "spanId": s, **({"parentSpanId": p} if p else {}), "name": "x", "kind": 2,
             "startTimeUnixNano": str(t0), "endTimeUnixNano": str(t1),
             "attributes": [{"key": k, "value": av(v)} for k, v in a.items()]}
            for t, s, p, t0, t1, a in spans]}]}]}).encode()


RES = {"service.name": "rag-service", "k8s.pod.uid": "0f1e2d3c-4b5a-6978-8796-a5b4c3d2e1f0", "process.pid": 4242}
SPANS = [
    (TID, "00f067aa0ba902b7", "", 1_700_000_000_000_000_000, 1_700_000_000_250_000_000,
     {"llm.slo.ttft_ms": 812.5, "client.port": 51000, "server.port": 443, "server.address": "10.0.0.7"}),
    (TID, "00f067aa0ba902b8", "00f067aa0ba902b7", 1_700_000_000_010_000_000, 1_700_000_000_020_000_000, {}),
    ("0af7651916cd43dd8448eb211c80319c", "b7ad6b7169203331", "", 1_700_000_000_500_000_000,
     1_700_000_000_900_000_000, {}),
]


def _mapper(cap=4):
    pods = Interner()
    return otlp.SpanMapper(otlp.GroupTable(cap), pods.id, node_id=3), pods


def _check(recs, pods):
    assert len(recs) == 2  # the child span is not a request span
    r = recs[0]
    assert r["trace_h"] == int(TID[16:], 16) == otlp.trace_hash(TID)
    assert r["ts_ns"] == SPANS[0][3] and abs(r["latency_ms"] - 250.0) < 1e-3
    assert abs(r["ttft_ms"] - 812.5) < 1e-4 and np.isnan(recs[1]["ttft_ms"])
    assert r["pid"] == 4242 and r["pod_id"] == pods.id(RES["k8s.pod.uid"]) == 1
    assert r["group_id"] == 0 and r["svc_id"] == 1 and r["node_id"] == 3
    # the address as the probes hold it (network-order bytes read little-endian, REF ipFromU32)
    assert records.ipv4_from_u32(0x0700000A) == "10.0.0.7"
    assert r["conn_h"] == records.conn_hash(51000, 443, 0x0700000A)
    assert r["span_h"] == 0x00F067AA0BA902B7
    assert recs[1]["conn_h"] == 0


def test_json_request_to_span_records():
    m, pods = _mapper()
    _check(m.records(otlp.parse_json(_request_json(RES, SPANS))), pods)


def test_proto_request_to_span_records():
    m, pods = _mapper()
    body = _request_pb(RES, [_span_pb(*s) for s in SPANS])
    _check(m.records(otlp.parse_proto(body)), pods)


def test_groups_overflow_into_last():
    g = otlp.GroupTable(2)
    assert [g.id(s) for s in ("a", "b", "c", "a", "d")] == [0, 1, 1, 0, 1]
    assert g.names == ["a", "b"]


def test_receiver_http_into_span_ring():
    from llm_slo_ebpf_toolkit_amd.runtime import load

    rt = load()
    ring = rt.HostRing(4, 64)
    m, pods = _mapper()
    rx = otlp.OtlpSpanReceiver("127.0.0.1:0", m, ring.push).start()
    try:
        for ctype, body in (("application/json", _request_json(RES, SPANS)),
                            ("application/x-protobuf", _request_pb(RES, [_span_pb(*s) for s in SPANS]))):
            req = urllib.request.Request(rx.endpoint, data=body, method="POST", headers={"Content-Type": ctype})
            assert urllib.request.urlopen(req, timeout=5).status == 200
        # the ring holds 4 records: a third request is accepted partially (ring full)
        req = urllib.request.Request(rx.endpoint, data=_request_json(RES, SPANS), method="POST",
                                     headers={"Content-Type": "application/json"})
        resp = json.loads(urllib.request.urlopen(req, timeout=5).read())
        assert resp["partialSuccess"]["rejectedSpans"] == "2"
        bad = urllib.request.Request(rx.endpoint, data=b"\xff\xff", method="POST",
                                     headers={"Content-Type": "application/x-protobuf"})
        try:
            urllib.request.urlopen(bad, timeout=5)
            raise AssertionError("malformed protobuf accepted")
        except urllib.error.HTTPError as e:
            assert e.code == 400
    finally:
        rx.stop()
    assert (rx.requests, rx.accepted, rx.dropped, rx.rejected) == (3, 4, 2, 1)
    assert ring.size == 4
    recs = ring.records_view()[: 4 * 64].view(records.SPAN)  # no wrap: the ring was empty
    _check(recs[:2], pods)
    _check(recs[2:4], pods)


def test_rag_service_spans_reach_the_ring():
    """The demo service's OTLP exporter -> the agent's receiver -> SPAN records carrying the
    request's trace hash, TTFT and the service's pod / pid."""
    import os

    from llm_slo_ebpf_toolkit_amd.demo.rag_service import RagService, StubBackend
    from llm_slo_ebpf_toolkit_amd.runtime import load

    rt = load()
    ring = rt.HostRing(64, 64)
    m, pods = _mapper()
    rx = otlp.OtlpSpanReceiver("127.0.0.1:0", m, ring.push).start()
    try:
        svc = RagService(StubBackend(), otlp_endpoint=rx.endpoint, resource={"k8s.pod.uid": RES["k8s.pod.uid"]},
                         early_ttft=False)  # (first-token records: tests/test_first_token.py)
        outs = [svc.chat({"prompt": f"why is ttft high {i}", "profile": "chat_short", "max_tokens": 2})
                for i in range(3)]
        svc.spans.flush()
    finally:
        rx.stop()
    assert ring.size == 3  # one request span per chat (retrieval / generation children stay out)
    buf = ring.records_view()[: 3 * 64].view(records.SPAN)
    by_trace = {int(r["trace_h"]): r for r in buf}
    for o in outs:
        r = by_trace[otlp.trace_hash(o["trace_id"])]
        assert abs(float(r["ttft_ms"]) - o["ttft_ms"]) < 1e-2
        assert r["pid"] == os.getpid() and r["pod_id"] == pods.id(RES["k8s.pod.uid"])
        assert r["group_id"] == 0
        # the retrieval child span's llm.slo.retrieval.* breakdown, folded into the request's record
        # (the breakdown is the plan's parts; the response's retrieval_ms the wall time around them)
        assert 0.0 < float(r["retr_ms"]) <= o["retrieval_ms"] + 0.5


def test_retrieval_breakdown_folds_into_the_request_span():
    """REF puts llm.slo.retrieval.{vectordb,network,dns}_ms on the chat.retrieval child span
    (demo/rag-service/main.go:393-397): the receiver sums them per trace onto the request's SPAN
    record, in the same export or from an earlier one (children end first); a trace without a
    breakdown carries 0 (no application evidence)."""
    m, _ = _mapper()
    retr = {"llm.slo.retrieval.vectordb_ms": 150.0, "llm.slo.retrieval.network_ms": 12.0,
            "llm.slo.retrieval.dns_ms": 6.5}
    child = (TID, "00f067aa0ba902b9", "00f067aa0ba902b7", 1_700_000_000_010_000_000, 1_700_000_000_180_000_000, retr)
    recs = m.records(otlp.parse_json(_request_json(RES, [child] + SPANS)))
    assert len(recs) == 2
    assert recs[0]["retr_ms"] == np.float32(168.5) and recs[1]["retr_ms"] == 0.0
    # the child in an earlier export than its request span
    m2, _ = _mapper()
    assert len(m2.records(otlp.parse_json(_request_json(RES, [child])))) == 0
    recs = m2.records(otlp.parse_json(_request_json(RES, SPANS)))
    assert recs[0]["retr_ms"] == np.float32(168.5)
    assert not m2._retr  # consumed
    # over protobuf, with junk parts ignored
    m3, _ = _mapper()
    bad = dict(retr, **{"llm.slo.retrieval.dns_ms": "n/a"})
    body = _request_pb(RES, [_span_pb(*(child[:5] + (bad,)))] + [_span_pb(*x) for x in SPANS])
    assert m3.records(otlp.parse_proto(body))[0]["retr_ms"] == np.float32(162.0)
    assert otlp.retrieval_ms({}) is None and otlp.retrieval_ms({"llm.slo.retrieval.vectordb_ms": -1.0}) is None
    # the pending table is bounded
    m4, _ = _mapper()
    m4.retrieval_cap = 4
    for i in range(10):
        m4.records(otlp.parse_json(_request_json(RES, [(f"{i:032x}",) + child[1:]])))
    assert len(m4._retr) == 4


def test_receiver_refuses_oversized_bodies_and_unlisted_peers():
    """The agent binds its receiver on the host network: a body over the cap is refused (413)
    before it is read, and with an allow-list a peer outside it gets 403."""
    import http.client

    from llm_slo_ebpf_toolkit_amd.runtime import load

    rt = load()
    ring = rt.HostRing(16, 64)
    m, _ = _mapper()
    body = _request_json(RES, SPANS)
    rx = otlp.OtlpSpanReceiver("127.0.0.1:0", m, ring.push, max_body=len(body) - 1).start()
    try:
        c = http.client.HTTPConnection(rx.addr[0], rx.addr[1], timeout=5)
        # the header announces 1 GiB; nothing past the headers is sent
        c.putrequest("POST", "/v1/traces")
        c.putheader("Content-Type", "application/json")
        c.putheader("Content-Length", str(1 << 30))
        c.endheaders()
        assert c.getresponse().status == 413
        c.close()
        req = urllib.request.Request(rx.endpoint, data=body, method="POST", headers={"Content-Type": "application/json"})
        try:
            urllib.request.urlopen(req, timeout=5)
            raise AssertionError("body over the cap accepted")
        except urllib.error.HTTPError as e:
            assert e.code == 413
    finally:
        rx.stop()
    assert ring.size == 0 and rx.refused == 2 and rx.requests == 0
    rx = otlp.OtlpSpanReceiver("127.0.0.1:0", m, ring.push, allow="10.0.0.0/8").start()
    try:
        req = urllib.request.Request(rx.endpoint, data=body, method="POST", headers={"Content-Type": "application/json"})
        try:
            urllib.request.urlopen(req, timeout=5)
            raise AssertionError("peer outside the allow-list accepted")
        except urllib.error.HTTPError as e:
            assert e.code == 403
    finally:
        rx.stop()
    assert ring.size == 0 and rx.refused == 1
    rx = otlp.OtlpSpanReceiver("127.0.0.1:0", m, ring.push, allow="127.0.0.0/8").start()
    try:
        req = urllib.request.Request(rx.endpoint, data=body, method="POST", headers={"Content-Type": "application/json"})
        assert urllib.request.urlopen(req, timeout=5).status == 200
    finally:
        rx.stop()
    assert ring.size == 2


def test_a_pods_service_is_bound_by_its_first_span():
    """the pod -> service table decides the service (and the GPU) a pod's kernel
    records belong to. A later span naming the same pod with another service is dropped, so a
    pod cannot move another pod's records to its service."""
    m, pods = _mapper()
    first = m.records(otlp.parse_json(_request_json(RES, SPANS)))
    assert len(first) == 2 and m.conflicts == 0
    other = dict(RES, **{"service.name": "intruder"})
    again = m.records(otlp.parse_json(_request_json(other, SPANS)))
    assert len(again) == 0 and m.conflicts >= 1
    upd = m.take_pod_updates()
    assert upd is not None and len(upd[0]) == 1  # one binding, from the first service


def test_span_naming_a_pod_must_come_from_its_address():
    groups = otlp.GroupTable(8)
    pods = Interner()
    uid = RES["k8s.pod.uid"]
    m = otlp.SpanMapper(groups, pods.id, 3, pod_ips=lambda: {"10.244.1.5": {uid}, "10.244.1.9": {"someone-else"}},
                        forwarders="10.244.7.0/24")
    body = otlp.parse_json(_request_json(RES, SPANS))
    assert len(m.records(body, "10.244.1.9")) == 0 and m.spoofed >= 1  # another pod's address
    assert len(m.records(body, "10.244.1.5")) > 0                      # its own address
    assert len(m.records(body, "10.244.7.3")) > 0                      # a trusted forwarder
    assert len(m.records(body, "192.168.9.9")) > 0                     # not a pod of this node


def test_local_addresses_from_fib_trie(tmp_path):
    from llm_slo_ebpf_toolkit_amd.collector import procfs

    d = tmp_path / "55" / "net"
    d.mkdir(parents=True)
    (d / "fib_trie").write_text("""Main:
  +-- 0.0.0.0/0 3 0 5
     |-- 0.0.0.0
        /0 universe UNICAST
     +-- 127.0.0.0/8 2 0 2
           |-- 127.0.0.1
              /32 host LOCAL
     +-- 10.244.1.0/24 2 0 2
           |-- 10.244.1.0
              /24 link UNICAST
           |-- 10.244.1.5
              /32 host LOCAL
        |-- 10.244.1.255
           /32 link BROADCAST
""")
    assert procfs.local_addresses(55, str(tmp_path)) == {"10.244.1.5"}
    assert procfs.pod_addresses({55: "uid-a", 56: "uid-a"}, str(tmp_path)) == {"10.244.1.5": {"uid-a"}}


def test_receiver_refuses_ambiguous_framing_and_keeps_a_connection_alive():
    """The receiver's header fast path: a duplicate Content-Length or a chunked body is refused
    (no guessing between framings), and an exporter's keep-alive connection carries request
    after request."""
    import http.client
    import socket

    from llm_slo_ebpf_toolkit_amd.runtime import load

    rt = load()
    ring = rt.HostRing(64, 64)
    m, _ = _mapper()
    body = _request_json(RES, SPANS)
    rx = otlp.OtlpSpanReceiver("127.0.0.1:0", m, ring.push).start()
    try:
        for extra in (f"Content-Length: {len(body)}\r\n", "Transfer-Encoding: chunked\r\n"):
            s = socket.create_connection(rx.addr, timeout=5)
            s.sendall((f"POST /v1/traces HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n"
                       f"Content-Length: {len(body)}\r\n{extra}\r\n").encode() + body)
            status = s.recv(4096).split(b"\r\n", 1)[0]
            s.close()
            assert status.split()[1] in (b"400", b"411"), status
        assert ring.size == 0
        c = http.client.HTTPConnection(rx.addr[0], rx.addr[1], timeout=5)
        for _ in range(3):
            c.request("POST", "/v1/traces", body=body, headers={"Content-Type": "application/json"})
            r = c.getresponse()
            assert r.status == 200 and r.read() == b"{}"
        c.close()
    finally:
        rx.stop()
    assert ring.size == 3 * len(m.records(otlp.parse_json(body)))
