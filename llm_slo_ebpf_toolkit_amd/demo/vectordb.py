"""Vector-DB stub for the RAG demo (config 3 of BASELINE.json: "demo/rag-service + vectordb").

REF's rag-service only sleeps for its vector-DB time (/root/reference/demo/rag-service/main.go:
641-671). This stub is a real network hop with real CPU work, so injected faults act on it the
way they would on a vector database: ``POST /search {"query": ..., "k": ...}`` embeds the query
(hashed bag of words), scores it against the corpus embeddings (dense dot products, numpy) and
returns the top-k documents. The RAG service talks to it over one keep-alive TCP connection
per worker thread, so its request spans carry that connection's tuple (client port, server
port, server address) and the node agent joins TCP-level kernel signals of the connection to
the requests (the pod+connection tier).

``POST /fault {"delay_ms": D}`` stalls every response by D ms until reset with 0: the latency a
lossy path adds to the connection (retransmission timeouts), for fault-injection runs on hosts
where ``tc netem`` needs privileges the harness does not have.

    python -m llm_slo_ebpf_toolkit_amd.demo.vectordb --bind 127.0.0.1:6333
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

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
DIM = 384


def embed(text: str, dim: int = DIM) -> np.ndarray:
    """Hashed bag-of-words embedding (unit norm)."""
    v = np.zeros(dim, dtype=np.float32)
    for w in text.lower().split():
        h = int.from_bytes(hashlib.blake2b(w.encode(), digest_size=8).digest(), "little")
        v[h % dim] += 1.0 if (h >> 63) & 1 else -1.0
    n = float(np.linalg.norm(v))
    return v / n if n else v


class VectorDB:
    def __init__(self, corpus_path: str = os.path.join(HERE, "fixtures", "corpus.json"), replicas: int = 256,
                 seed: int = 42):
        with open(corpus_path) as fh:
            docs = json.load(fh)
        rng = np.random.default_rng(seed)
        # the corpus plus perturbed replicas: a search scans ~len(corpus) * replicas vectors
        self.titles = [d["title"] for d in docs for _ in range(replicas)]
        base = np.stack([embed(d["title"] + " " + d.get("text", d.get("content", ""))) for d in docs])
        noise = rng.normal(0, 0.05, size=(len(docs), replicas, DIM)).astype(np.float32)
        self.matrix = (base[:, None, :] + noise).reshape(-1, DIM)
        self.searches = 0
        self.delay_ms = 0.0
        self._lock = threading.Lock()

    def search(self, query: str, k: int = 4):
        q = embed(query)
        scores = self.matrix @ q
        top = np.argpartition(-scores, min(k, len(scores) - 1))[:k]
        top = top[np.argsort(-scores[top])]
        with self._lock:
            self.searches += 1
        return [{"title": self.titles[i], "score": float(scores[i])} for i in top]

    def handler(self):
        db = self

        class H(http.server.BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"  # keep-alive: one connection per client thread

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
                self._json(200 if self.path == "/healthz" else 404, {"status": "ok", "searches": db.searches})

            def do_POST(self):
                if self.path == "/fault":
                    n = int(self.headers.get("Content-Length") or 0)
                    try:
                        db.delay_ms = max(0.0, float(json.loads(self.rfile.read(n) or b"{}").get("delay_ms", 0)))
                    except (ValueError, TypeError, AttributeError):
                        self._json(400, {"error": "delay_ms must be a number"})
                        return
                    self._json(200, {"delay_ms": db.delay_ms})
                    return
                if self.path != "/search":
                    self._json(404, {"error": "not found"})
                    return
                n = int(self.headers.get("Content-Length") or 0)
                try:
                    req = json.loads(self.rfile.read(n) or b"{}")
                except json.JSONDecodeError:
                    self._json(400, {"error": "invalid json"})
                    return
                t0 = time.perf_counter()
                hits = db.search(str(req.get("query", "")), int(req.get("k", 4)))
                if db.delay_ms:
                    time.sleep(db.delay_ms / 1000.0)
                self._json(200, {"hits": hits, "took_ms": round(1e3 * (time.perf_counter() - t0), 3)})

        return H

    def serve(self, bind: str):
        host, port = bind.rsplit(":", 1)
        httpd = http.server.ThreadingHTTPServer((host or "127.0.0.1", int(port)), self.handler())
        httpd.daemon_threads = True
        threading.Thread(target=httpd.serve_forever, daemon=True).start()
        return httpd


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="vector-DB stub for the RAG demo")
    ap.add_argument("--bind", default="127.0.0.1:6333")
    ap.add_argument("--replicas", type=int, default=256)
    a = ap.parse_args(argv)
    httpd = VectorDB(replicas=a.replicas).serve(a.bind)
    print(f"vectordb listening on {a.bind}", flush=True)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        httpd.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
