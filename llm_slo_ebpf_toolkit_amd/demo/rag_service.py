"""Demo RAG chat service (REF demo/rag-service/main.go, re-built in Python).

``POST /chat`` {"prompt", "profile", "seed", "max_tokens", "stream", "request_id"}:

1. a deterministic retrieval plan per (profile, prompt, seed) -- DNS, network and vector-DB
   waits, documents from ``fixtures/corpus.json``;
2. span ``chat.retrieval`` with ``llm.slo.retrieval.*`` attributes, DNS enrichment of the
   request span through the correlator (tier + confidence -> ``llm_slo_correlation_total``);
3. span ``chat.generation`` from the backend: ``stub`` (seeded token list, paced) or
   ``llama`` (the random-init Llama on the local MI355X: real prefill + decode, so TTFT
   carries GPU queueing / HBM / RCCL effects);
4. streaming NDJSON (``{"token": ...}`` lines then a summary) or one JSON document.

Prometheus on ``--metrics-bind``: ``llm_slo_ttft_ms``, ``llm_slo_tokens_per_sec``,
``llm_slo_retrieval_{vectordb,network,dns}_ms`` histograms, ``llm_slo_requests_total``,
``llm_slo_correlation_total`` -- and, closing a REF gap (the cdgate queries
reference series nobody emitted), ``llm_slo_errors_total`` and ``llm_slo_burn_rate``
(error-budget burn over a sliding window against a 99 % objective).
Traces: OTLP/HTTP JSON (``/v1/traces``) when ``--otlp-endpoint`` is set, batched.
"""

from __future__ import annotations

import argparse
import collections
import hashlib
import http.server
import json
import os
import random
import sys
import threading
import time
import urllib.request
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

from ..contracts import semconv
from ..correlation.correlator import Correlator
from ..correlation.match import SignalRef, SpanRef
from ..export.prometheus import MetricsServer, Registry
from ..utils.timeutil import MS

HERE = os.path.dirname(os.path.abspath(__file__))
VOCAB = ("reliability", "signal", "trace", "kernel", "latency", "attribution", "dns", "retrieval", "throughput",
         "incident", "confidence", "evidence", "burn", "slo", "token", "scheduler", "gpu", "xgmi")


@dataclass
class Plan:
    dns_ms: float
    network_ms: float
    vectordb_ms: float
    warmup_ms: int
    cadence_ms: int
    docs: int


def prompt_hash(prompt: str) -> int:
    return int.from_bytes(hashlib.blake2b(prompt.encode(), digest_size=4).digest(), "little")


def plan_for(profile: str, prompt: str, seed: int) -> Plan:
    """Same ranges per profile as REF planForRequest (demo/rag-service/main.go:673-707)."""
    r = random.Random(seed + prompt_hash(prompt))
    if profile == "chat_short":
        return Plan(2 + r.randrange(4), 4 + r.randrange(8), 10 + r.randrange(20), 25 + r.randrange(15),
                    25 + r.randrange(10), 2 + r.randrange(2))
    if profile == "context_long":
        return Plan(8 + r.randrange(8), 15 + r.randrange(20), 70 + r.randrange(80), 50 + r.randrange(30),
                    45 + r.randrange(20), 4 + r.randrange(2))
    return Plan(5 + r.randrange(8), 10 + r.randrange(14), 35 + r.randrange(45), 30 + r.randrange(20),
                30 + r.randrange(15), 3 + r.randrange(2))


def stub_tokens(prompt: str, max_tokens: int, seed: int) -> List[str]:
    max_tokens = min(max(1, max_tokens), 256)
    r = random.Random(seed + prompt_hash(prompt))
    out = [t for t in prompt.split() if t.strip()][:max_tokens]
    while len(out) < max_tokens:
        out.append(VOCAB[r.randrange(len(VOCAB))])
    return out


class StubBackend:
    name = "stub"

    def generate(self, prompt: str, max_tokens: int, seed: int, plan: Plan, emit, on_start=None) -> Dict[str, float]:
        toks = stub_tokens(prompt, max_tokens, seed)
        if on_start:
            on_start()
        t0 = time.perf_counter()
        time.sleep(plan.warmup_ms / 1000.0)
        ttft = time.perf_counter() - t0
        for i, t in enumerate(toks):
            if i:
                time.sleep(plan.cadence_ms / 1000.0)
            emit(t)
        total = time.perf_counter() - t0
        return {"ttft_s": ttft, "total_s": total, "tokens": len(toks)}


class LlamaBackend:
    """Random-init Llama on the local GPU; token ids are rendered as vocabulary words."""
    name = "llama"

    def __init__(self, preset: str = "1b", device: str = "cuda"):
        import torch

        from ..models.llama import build

        self.torch = torch
        self.model = build(preset, device)
        self.lock = threading.Lock()
        self.device = device

    def generate(self, prompt: str, max_tokens: int, seed: int, plan: Plan, emit, on_start=None) -> Dict[str, float]:
        torch = self.torch
        ids = [prompt_hash(w) % self.model.cfg.vocab for w in prompt.split()] or [1]
        x = torch.tensor([ids], device=self.device)
        with self.lock:  # one request on the GPU at a time (the demo is latency-oriented)
            if on_start:
                on_start()
            r = self.model.generate(x, max(1, min(max_tokens, 256)),
                                    on_token=lambda t: emit(VOCAB[int(t.item()) % len(VOCAB)]))
        return {"ttft_s": r["ttft_ms"] / 1e3, "total_s": r["total_ms"] / 1e3, "tokens": r["new_tokens"]}


class GpuTraceTag:
    """Tags the GPU work of a request with its trace: when the rocprofiler-sdk tool
    (probes/rocprof, libmislo_rocprof.so) is loaded into this process, the kernels the calling
    thread enqueues carry the request's trace hash (the OTLP receiver's rule: low 64 bits of the
    W3C id), so the agent joins them to the request's spans through the trace tier. A no-op
    without the tool."""

    def __init__(self):
        self._set = None
        self._resolved = False

    def _resolve(self) -> None:
        # the tool is loaded when the HIP runtime starts (first GPU use), so resolve lazily
        self._resolved = True
        try:
            with open("/proc/self/maps") as f:
                path = next((ln.split()[-1] for ln in f if ln.rstrip().endswith("libmislo_rocprof.so")), None)
            if path:
                import ctypes

                fn = ctypes.CDLL(path, mode=os.RTLD_NOLOAD | os.RTLD_NOW).mislo_rocprof_set_trace
                fn.argtypes, fn.restype = [ctypes.c_uint64], None
                self._set = fn
        except (OSError, AttributeError):
            self._set = None

    @property
    def active(self) -> bool:
        if not self._resolved:
            self._resolve()
        return self._set is not None

    def set(self, trace_id: str) -> None:
        from ..collector.otlp import trace_hash

        self.set_hash(trace_hash(trace_id) if trace_id else 0)

    def set_hash(self, h: int) -> None:
        """The trace hash itself (another process computed it: a TP rank tags its shard's kernels
        with the request rank 0 received)."""
        if not self._resolved:
            self._resolve()
        if self._set is not None:
            self._set(int(h) & 0xFFFFFFFFFFFFFFFF)


class SpanExporter:
    """Batched OTLP/HTTP JSON trace export (chat.request / chat.retrieval / chat.generation):
    a batch goes out when it holds ``max_batch`` spans or its oldest span is ``max_delay_s`` old
    (the OTel batch processor's schedule delay), so spans reach the agent's windows promptly."""

    def __init__(self, endpoint: str, service: str = "rag-service", max_batch: int = 64, resource=None,
                 max_delay_s: float = 0.2):
        self.endpoint, self.service, self.max_batch = endpoint, service, max_batch
        self.max_delay_s = max_delay_s
        self.buf: List[dict] = []
        self.lock = threading.Lock()
        self._wake = threading.Event()
        if endpoint and max_delay_s > 0:
            threading.Thread(target=self._flusher, name="span-flush", daemon=True).start()
        # resource identity the agent's OTLP receiver maps onto its pod / process ids
        # (collector/otlp.py): pod uid / name and node from the downward API, this process's pid
        res = {"service.name": service, "process.pid": os.getpid(),
               "k8s.pod.uid": os.environ.get("POD_UID", ""), "k8s.pod.name": os.environ.get("POD_NAME", ""),
               "k8s.node.name": os.environ.get("NODE_NAME", "")}
        res.update(resource or {})
        self.resource = [{"key": k, "value": self._val(v)} for k, v in res.items() if v not in ("", None)]

    @staticmethod
    def _val(v):
        if isinstance(v, bool):
            return {"boolValue": v}
        if isinstance(v, int):
            return {"intValue": str(v)}
        if isinstance(v, float):
            return {"doubleValue": v}
        return {"stringValue": str(v)}

    @staticmethod
    def span(trace_id: str, span_id: str, parent: str, name: str, t0: int, t1: int, attrs: Dict[str, object]):
        d = {"traceId": trace_id, "spanId": span_id, "name": name, "kind": 2, "startTimeUnixNano": str(t0),
             "endTimeUnixNano": str(t1),
             "attributes": [{"key": k, "value": SpanExporter._val(v)} for k, v in attrs.items()]}
        if parent:
            d["parentSpanId"] = parent
        return d

    def add(self, spans: List[dict], urgent: bool = False) -> None:
        """Queue spans; ``urgent``: the flusher sends them now instead of at the batch delay
        (without blocking the caller -- the request thread)."""
        if not self.endpoint:
            return
        with self.lock:
            self.buf += spans
            if len(self.buf) < self.max_batch:
                if urgent:
                    self._wake.set()
                return
            batch, self.buf = self.buf, []
        self._post(batch)

    def flush(self) -> None:
        with self.lock:
            batch, self.buf = self.buf, []
        if batch:
            self._post(batch)

    def _flusher(self) -> None:
        while True:
            self._wake.wait(self.max_delay_s)
            self._wake.clear()
            self.flush()

    def _post(self, spans: List[dict]) -> None:
        body = {"resourceSpans": [{"resource": {"attributes": self.resource},
                                   "scopeSpans": [{"scope": {"name": "rag-service"}, "spans": spans}]}]}
        req = urllib.request.Request(self.endpoint, data=json.dumps(body).encode(), method="POST",
                                     headers={"Content-Type": "application/json"})
        try:
            urllib.request.urlopen(req, timeout=5).read()
        except Exception as exc:  # noqa: BLE001 - tracing must never fail a request
            print(f"trace export failed: {exc}", file=sys.stderr)


class BurnRate:
    """Error-budget burn rate over a sliding window: error_ratio / (1 - objective)."""

    def __init__(self, objective: float = 0.99, window_s: float = 300.0):
        self.objective, self.window_s = objective, window_s
        self.events = collections.deque()

    def observe(self, ok: bool, now: Optional[float] = None) -> float:
        now = time.monotonic() if now is None else now
        self.events.append((now, ok))
        while self.events and self.events[0][0] < now - self.window_s:
            self.events.popleft()
        n = len(self.events)
        errs = sum(1 for _, o in self.events if not o)
        return (errs / n) / (1.0 - self.objective) if n else 0.0


class VectorDBClient:
    """Keep-alive HTTP client of the vector-DB stub (demo/vectordb.py), one TCP connection per
    worker thread: a request's span carries its connection's tuple, so TCP-level kernel signals
    of that connection join the request (pod + connection tier)."""

    def __init__(self, url: str, timeout_s: float = 10.0):
        from urllib.parse import urlparse

        u = urlparse(url)
        self.host, self.port, self.timeout = u.hostname or "127.0.0.1", int(u.port or 80), timeout_s
        self._tls = threading.local()

    def _conn(self):
        import http.client

        c = getattr(self._tls, "conn", None)
        if c is None:
            c = http.client.HTTPConnection(self.host, self.port, timeout=self.timeout)
            c.connect()
            self._tls.conn = c
        return c

    def search(self, query: str, k: int) -> Tuple[List[str], Dict[str, object]]:
        """(titles, connection attributes: client.port / server.port / server.address)."""
        for attempt in (0, 1):
            c = self._conn()
            try:
                body = json.dumps({"query": query, "k": k}).encode()
                c.request("POST", "/search", body=body, headers={"Content-Type": "application/json"})
                out = json.loads(c.getresponse().read())
                lip, lport = c.sock.getsockname()[:2]
                rip, rport = c.sock.getpeername()[:2]
                return [h["title"] for h in out["hits"]], {"client.port": int(lport), "server.port": int(rport),
                                                           "server.address": rip}
            except (OSError, ValueError):
                c.close()
                self._tls.conn = None
                if attempt:
                    raise
        return [], {}


class RagService:
    def __init__(self, backend, corpus_path: str = os.path.join(HERE, "fixtures", "corpus.json"),
                 otlp_endpoint: str = "", node: str = "demo-node", pod: str = "demo-rag-service", resource=None,
                 vectordb_url: str = "", early_ttft: bool = True):
        self.backend = backend
        # export the TTFT SLI when the first token is out (a chat.first_token span,
        # llm.slo.ttft_early), not only on the request span at the end: an SLO breach reaches the
        # agent's window it happened in (collector/otlp.py counts each request once)
        self.early_ttft = early_ttft
        self.vdb = VectorDBClient(vectordb_url) if vectordb_url else None
        with open(corpus_path) as fh:
            self.docs = json.load(fh)
        self.corr = Correlator()
        self.node, self.pod = node, pod
        self.spans = SpanExporter(otlp_endpoint, resource=resource)
        self.gpu_tag = GpuTraceTag()
        self.burn = BurnRate()
        r = self.registry = Registry()
        ms = (5, 10, 25, 50, 100, 200, 400, 800, 1600, 3200)
        self.m_ttft = r.histogram("llm_slo_ttft_ms", "Time to first token (ms).", ms)
        self.m_tps = r.histogram("llm_slo_tokens_per_sec", "Decode tokens per second.", (1, 5, 10, 20, 40, 80, 160, 320))
        self.m_vdb = r.histogram("llm_slo_retrieval_vectordb_ms", "Vector DB time (ms).", ms)
        self.m_net = r.histogram("llm_slo_retrieval_network_ms", "Retrieval network time (ms).", ms)
        self.m_dns = r.histogram("llm_slo_retrieval_dns_ms", "Retrieval DNS time (ms).", ms)
        self.m_req = r.counter("llm_slo_requests_total", "Chat requests by status and profile.", ("status", "profile"))
        self.m_err = r.counter("llm_slo_errors_total", "Failed chat requests by profile.", ("profile",))
        self.m_corr = r.counter("llm_slo_correlation_total", "DNS correlation decisions by tier and enrichment.",
                                ("tier", "enriched"))
        self.m_burn = r.gauge("llm_slo_burn_rate", "Error-budget burn rate (5 min window, 99% objective).")

    def _fail(self, profile: str) -> None:
        self.m_req.inc(1, "error", profile)
        self.m_err.inc(1, profile)
        self.m_burn.set(self.burn.observe(False))

    def chat(self, req: dict, emit=None) -> dict:
        prompt = (req.get("prompt") or "").strip()
        if not prompt:
            self.m_req.inc(1, "bad_request", "unknown")
            raise ValueError("prompt is required")
        profile = req.get("profile") or "rag_medium"
        seed = int(req.get("seed") or 42)
        max_tokens = int(req.get("max_tokens") or 64)
        rid = req.get("request_id") or f"req-{time.time_ns()}"
        trace_id = hashlib.blake2b(rid.encode(), digest_size=16).hexdigest()
        root, rsp, gsp = (hashlib.blake2b(f"{rid}/{k}".encode(), digest_size=8).hexdigest() for k in "rxg")
        t_req = time.time_ns()
        plan = plan_for(profile, prompt, seed)
        rnd = random.Random(seed + prompt_hash(prompt))
        docs = sorted(d["title"] for d in rnd.sample(self.docs, min(plan.docs, len(self.docs))))
        t_r0 = time.time_ns()
        conn_attrs: Dict[str, object] = {}
        if self.vdb is not None:  # a real vector-DB hop; DNS and network stay the plan's
            for wait in (plan.dns_ms, plan.network_ms):
                time.sleep(wait / 1000.0)
            t_v = time.time_ns()
            docs, conn_attrs = self.vdb.search(prompt, plan.docs)
            vdb_ms = (time.time_ns() - t_v) / MS
        else:
            for wait in (plan.dns_ms, plan.network_ms, plan.vectordb_ms):
                time.sleep(wait / 1000.0)
            vdb_ms = plan.vectordb_ms
        t_r1 = time.time_ns()
        # spans leave as an OTel SDK's batch processor sends them, as they end: the retrieval span
        # now, ahead of the request's first token (its breakdown reaches the agent with the
        # first-token record instead of at the request's end)
        self.spans.add([SpanExporter.span(trace_id, rsp, root, "chat.retrieval", t_r0, t_r1, {
            semconv.ATTR_RETRIEVAL_VECTORDB: float(vdb_ms),
            semconv.ATTR_RETRIEVAL_NETWORK_MS: float(plan.network_ms),
            semconv.ATTR_RETRIEVAL_DNS_MS: float(plan.dns_ms), "retrieval.selected_docs": len(docs)})])
        span = SpanRef(trace_id=trace_id, service="rag-service", node=self.node, pod=self.pod, pid=os.getpid(),
                       timestamp=t_req)
        sig = SignalRef(signal="dns_latency_ms", trace_id=trace_id, service="rag-service", node=self.node,
                        pod=self.pod, pid=os.getpid(), timestamp=time.time_ns(), value=float(plan.dns_ms))
        attrs, decision = self.corr.enrich_dns_attributes(None, span, sig)
        if decision.matched:
            enriched = "true" if decision.confidence >= self.corr.enrichment_threshold else "false"
            self.m_corr.inc(1, decision.tier, enriched)
        tokens: List[str] = []

        def on_tok(t):
            tokens.append(t)
            if len(tokens) == 1 and self.early_ttft:
                # the request span's TTFT definition (retrieval + the backend's time to its first
                # token, a wait for the backend's lock excluded), known now instead of at the end;
                # with the request's connection, so the record joins the pod+conn tier as well
                t_ft = time.time_ns()
                ttft_now = (t_r1 - t_req) / MS + (t_ft - t_gen[0]) / MS
                ft_attrs = {semconv.ATTR_SLO_TTFT_MS: ttft_now, semconv.ATTR_SLO_TTFT_EARLY: True}
                ft_attrs.update(conn_attrs)
                self.spans.add([SpanExporter.span(
                    trace_id, hashlib.blake2b(f"{rid}/f".encode(), digest_size=8).hexdigest(), root, "chat.first_token",
                    t_req, t_ft, ft_attrs)], urgent=True)
            if emit:
                emit({"token": t, "index": len(tokens) - 1})

        t_gen = [time.time_ns()]

        def on_start():
            t_gen[0] = time.time_ns()

        self.gpu_tag.set(trace_id)  # this request's kernels carry its trace
        try:
            g = self.backend.generate(prompt, max_tokens, seed, plan, on_tok, on_start=on_start)
        except Exception:
            self._fail(profile)
            raise
        finally:
            self.gpu_tag.set("")
        t_end = time.time_ns()
        ret_ms = (t_r1 - t_r0) / MS
        ttft_ms = (t_r1 - t_req) / MS + g["ttft_s"] * 1e3
        dec_s = max(g["total_s"] - g["ttft_s"], 1e-9)
        tps = (g["tokens"] - 1) / dec_s if g["tokens"] > 1 else float(g["tokens"])
        self.m_ttft.observe(ttft_ms)
        self.m_tps.observe(tps)
        self.m_vdb.observe(vdb_ms)
        self.m_net.observe(plan.network_ms)
        self.m_dns.observe(plan.dns_ms)
        self.m_req.inc(1, "ok", profile)
        self.m_burn.set(self.burn.observe(True))
        root_attrs = {"request.id": rid, "llm.profile": profile, "llm.seed": seed, "llm.backend": self.backend.name,
                      semconv.ATTR_SLO_TTFT_MS: ttft_ms, semconv.ATTR_SLO_TOKENS_PER_SEC: tps}
        root_attrs.update({k: float(v) for k, v in (attrs or {}).items()})
        root_attrs.update(conn_attrs)
        if decision.tier:
            root_attrs["llm.ebpf.correlation_tier"] = decision.tier
        # as they end: the generation before the request
        self.spans.add([
            SpanExporter.span(trace_id, gsp, root, "chat.generation", t_r1, t_end, {"llm.tokens.count": g["tokens"]}),
            SpanExporter.span(trace_id, root, "", "chat.request", t_req, t_end, root_attrs),
        ])
        return {"request_id": rid, "trace_id": trace_id, "profile": profile, "tokens": tokens, "documents": docs,
                "ttft_ms": round(ttft_ms, 3), "tokens_per_sec": round(tps, 3), "retrieval_ms": round(ret_ms, 3),
                "correlation": {"tier": decision.tier, "confidence": decision.confidence},
                "attributes": attrs or {}, "retrieval_conn": conn_attrs}

    def handler(self):
        svc = self

        class H(http.server.BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):
                pass

            def _json(self, code, obj):
                b = json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(b)))
                self.end_headers()
                self.wfile.write(b)

            def do_GET(self):
                if self.path == "/healthz":
                    self._json(200, {"status": "ok"})
                else:
                    self._json(404, {"error": "not found"})

            def do_POST(self):
                if self.path != "/chat":
                    self._json(404, {"error": "not found"})
                    return
                n = int(self.headers.get("Content-Length") or 0)
                try:
                    req = json.loads(self.rfile.read(n) or b"{}")
                except json.JSONDecodeError:
                    svc.m_req.inc(1, "bad_request", "unknown")
                    self._json(400, {"error": "invalid json body"})
                    return
                if req.get("stream"):
                    self.send_response(200)
                    self.send_header("Content-Type", "application/x-ndjson")
                    self.send_header("Transfer-Encoding", "chunked")
                    self.end_headers()

                    def emit(d):
                        line = (json.dumps(d) + "\n").encode()
                        self.wfile.write(f"{len(line):x}\r\n".encode() + line + b"\r\n")
                        self.wfile.flush()

                    try:
                        out = svc.chat(req, emit)
                        out.pop("tokens", None)
                        emit({"done": True, **out})
                    except ValueError as exc:
                        emit({"error": str(exc)})
                    except Exception as exc:  # noqa: BLE001
                        emit({"error": f"generation failed: {exc}"})
                    self.wfile.write(b"0\r\n\r\n")
                    return
                try:
                    self._json(200, svc.chat(req))
                except ValueError as exc:
                    self._json(400, {"error": str(exc)})
                except Exception as exc:  # noqa: BLE001
                    self._json(502, {"error": f"generation failed: {exc}"})

        return H

    def serve(self, bind: str = "127.0.0.1:8080", metrics_bind: str = "127.0.0.1:9464"):
        host, port = bind.rsplit(":", 1)
        httpd = http.server.ThreadingHTTPServer((host or "0.0.0.0", int(port)), self.handler())
        metrics = MetricsServer(self.registry, metrics_bind).start() if metrics_bind else None
        t = threading.Thread(target=httpd.serve_forever, daemon=True)
        t.start()
        return httpd, metrics


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="demo RAG chat service")
    ap.add_argument("--bind", default="0.0.0.0:8080")
    ap.add_argument("--metrics-bind", default="0.0.0.0:9464")
    ap.add_argument("--backend", default=os.environ.get("LLM_BACKEND", "stub"), choices=("stub", "llama"))
    ap.add_argument("--llama-preset", default="1b")
    ap.add_argument("--otlp-endpoint", default=os.environ.get("OTEL_EXPORTER_OTLP_TRACES_ENDPOINT", ""))
    ap.add_argument("--early-ttft", type=int, default=1, help="1: export each request's TTFT when its first token "
                                                                "is out (chat.first_token), not only at its end")
    ap.add_argument("--vectordb-url", default=os.environ.get("VECTORDB_URL", ""),
                    help="vector-DB stub (demo/vectordb.py) to search over a keep-alive connection")
    a = ap.parse_args(argv)
    backend = LlamaBackend(a.llama_preset) if a.backend == "llama" else StubBackend()
    svc = RagService(backend, otlp_endpoint=a.otlp_endpoint, vectordb_url=a.vectordb_url, early_ttft=bool(a.early_ttft))
    httpd, _ = svc.serve(a.bind, a.metrics_bind)
    print(f"rag-service listening on {a.bind} (backend={backend.name})", flush=True)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        httpd.shutdown()
        svc.spans.flush()
    return 0


if __name__ == "__main__":
    sys.exit(main())
