"""Tensor-parallel LLM server for config 4 (BASELINE.json: "8xMI355X TP inference under
RCCL-latency + CPU-steal injection").

One process per GPU (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT from the launcher,
torch.distributed over RCCL): every rank holds its tensor-parallel shard of the Llama model
(parallel/tensor.py: two RCCL all-reduces per layer over xGMI). Rank 0 serves ``POST /chat`` and
``GET /healthz``; each request's prompt goes to every rank with one broadcast, all ranks decode in
lock step, rank 0 answers with the TTFT and exports the request's spans over OTLP (the same
exporter and resource identity as the RAG demo, so the node agent joins the ranks' GPU signals --
kernel queue delay, RCCL collective time, xGMI latency from the rocprofiler tool each rank loads --
to the requests).

    python -m llm_slo_ebpf_toolkit_amd.demo.tp_server --preset 7b --bind 127.0.0.1:8090  # under a launcher
"""

from __future__ import annotations

import argparse
import hashlib
import http.server
import json
import os
import sys
import threading
import time

STOP = -1


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="tensor-parallel LLM server (config 4)")
    ap.add_argument("--preset", default="7b")
    ap.add_argument("--bind", default="127.0.0.1:8090")
    ap.add_argument("--otlp-endpoint", default=os.environ.get("OTEL_EXPORTER_OTLP_TRACES_ENDPOINT", ""))
    ap.add_argument("--max-new", type=int, default=16)
    ap.add_argument("--early-ttft", type=int, default=1, help="1: export each request's TTFT when its first token "
                                                                "is out (chat.first_token), not only at its end")
    ap.add_argument("--device", default="cuda", choices=("cuda", "cpu"), help="cpu: the gloo rehearsal (tests)")
    a = ap.parse_args(argv)

    import torch
    import torch.distributed as dist

    from ..contracts import semconv
    from ..parallel.tensor import build_tp
    from .rag_service import VOCAB, GpuTraceTag, SpanExporter, prompt_hash

    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", rank))
    if a.device == "cuda":
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if world > 1:
        if a.device == "cuda":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    model = build_tp(a.preset, rank, world, device=dev, dtype=torch.bfloat16 if a.device == "cuda" else torch.float32)
    hdr = torch.zeros(3, dtype=torch.int64, device=dev)   # [prompt length | STOP, max_new, trace hash]
    buf = torch.zeros(256, dtype=torch.int64, device=dev)

    tag = GpuTraceTag()

    def step(ids, max_new, on_token=None):
        """One request on every rank (rank 0 calls it with the ids, the others get them). Every
        rank tags its kernels with the request's trace, so the agent joins all shards' GPU
        signals to the request."""
        if world > 1:
            dist.broadcast(hdr, 0)
            n = int(hdr[0].item())
            if n == STOP:
                return None
            dist.broadcast(buf[:n], 0)
            x = buf[:n].view(1, n).clone()
            max_new = int(hdr[1].item())
            if rank:
                tag.set_hash(int(hdr[2].item()))
        else:
            x = ids
        try:
            return model.generate(x, max_new, on_token=on_token)
        finally:
            if rank:
                tag.set_hash(0)

    if rank != 0:
        while step(None, 0) is not None:
            pass
        dist.destroy_process_group()
        return 0

    from ..collector.otlp import trace_hash

    spans = SpanExporter(a.otlp_endpoint, service="llm-tp", resource={"llm.tp.world_size": world})
    lock = threading.Lock()
    stats = {"requests": 0}

    def chat(req):
        prompt = (req.get("prompt") or "").strip() or "hello"
        rid = req.get("request_id") or f"req-{time.time_ns()}"
        max_new = max(1, min(int(req.get("max_tokens") or a.max_new), 128))
        toks = [prompt_hash(w) % model.cfg.vocab for w in prompt.split()][:256] or [1]
        trace = hashlib.blake2b(rid.encode(), digest_size=16).hexdigest()
        root = hashlib.blake2b(f"{rid}/r".encode(), digest_size=8).hexdigest()
        t_arrive = time.time_ns()
        with lock:  # requests are serialised: every rank runs the same one
            # the span is the request's service (what TTFT is measured over), its wait for the
            # lock an attribute: the agent joins signals near the span's start, and a start
            # several queued requests back would fall outside the records it still holds
            t0 = time.time_ns()
            ids = torch.tensor([toks], dtype=torch.int64, device=dev)
            if world > 1:
                th = trace_hash(trace)
                hdr[0], hdr[1], hdr[2] = len(toks), max_new, th - (1 << 64) if th >= 1 << 63 else th
                buf[:len(toks)] = ids[0]
            tag.set(trace)
            first = []

            def on_token(_tok):  # the TTFT SLI as the first token is out (collector/otlp.py counts once)
                if not first:
                    first.append(time.time_ns())
                    spans.add([SpanExporter.span(
                        trace, hashlib.blake2b(f"{rid}/f".encode(), digest_size=8).hexdigest(), root,
                        "chat.first_token", t0, first[0],
                        {semconv.ATTR_SLO_TTFT_MS: (first[0] - t0) / 1e6, semconv.ATTR_SLO_TTFT_EARLY: True})],
                        urgent=True)

            try:
                r = step(ids, max_new, on_token if a.early_ttft else None)
            finally:
                tag.set("")
        t1 = time.time_ns()
        stats["requests"] += 1
        spans.add([SpanExporter.span(trace, root, "", "chat.request", t0, t1, {
            "request.id": rid, "llm.tp.world_size": world, semconv.ATTR_SLO_TTFT_MS: r["ttft_ms"],
            semconv.ATTR_SLO_TOKENS_PER_SEC: r["tokens_per_s"], "llm.queue_ms": round((t0 - t_arrive) / 1e6, 3)})])
        return {"request_id": rid, "trace_id": trace, "ttft_ms": round(r["ttft_ms"], 3),
                "tokens_per_sec": round(r["tokens_per_s"], 3), "tokens": [VOCAB[i % len(VOCAB)] for i in range(max_new)]}

    class H(http.server.BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def log_message(self, *x):
            pass

        def _json(self, code, obj):
            b = json.dumps(obj).encode()
            self.send_response(code)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(b)))
            self.end_headers()
            self.wfile.write(b)

        def do_GET(self):
            self._json(200 if self.path == "/healthz" else 404, {"status": "ok", "world": world, **stats})

        def do_POST(self):
            if self.path != "/chat":
                self._json(404, {"error": "not found"})
                return
            n = int(self.headers.get("Content-Length") or 0)
            try:
                self._json(200, chat(json.loads(self.rfile.read(n) or b"{}")))
            except (ValueError, KeyError) as exc:
                self._json(400, {"error": str(exc)})

    host, port = a.bind.rsplit(":", 1)
    httpd = http.server.ThreadingHTTPServer((host, int(port)), H)
    httpd.daemon_threads = True
    th = threading.Thread(target=httpd.serve_forever, daemon=True)
    th.start()
    print(f"tp-server rank 0 of {world} listening on {a.bind}", flush=True)
    import signal as _signal

    done = threading.Event()
    for s in (_signal.SIGTERM, _signal.SIGINT):
        _signal.signal(s, lambda *_: done.set())
    done.wait()
    httpd.shutdown()
    spans.flush()
    if world > 1:
        with lock:
            hdr[0] = STOP
            dist.broadcast(hdr, 0)
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
