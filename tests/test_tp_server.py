"""The config-4 TP server (demo/tp_server.py) on the CPU: two ranks over gloo hold their tensor-
parallel shards, rank 0 serves /chat, each request runs on both ranks in lock step, and SIGTERM
stops both (rank 0 broadcasts the stop)."""

import json
import os
import signal
import socket
import subprocess
import sys
import time
import urllib.request

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(240)
def test_two_rank_tp_server_serves_requests_and_stops():
    http_port, master = _port(), _port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(master), PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, "-m", "llm_slo_ebpf_toolkit_amd.demo.tp_server", "--preset", "tiny",
                                       "--device", "cpu", "--bind", f"127.0.0.1:{http_port}", "--otlp-endpoint", ""],
                                      cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    try:
        t0 = time.time()
        while True:
            try:
                h = json.loads(urllib.request.urlopen(f"http://127.0.0.1:{http_port}/healthz", timeout=2).read())
                break
            except OSError:
                assert all(p.poll() is None for p in procs), [p.stdout.read() for p in procs]
                assert time.time() - t0 < 180
                time.sleep(0.5)
        assert h["world"] == 2
        for i in range(3):
            req = urllib.request.Request(f"http://127.0.0.1:{http_port}/chat", method="POST",
                                         data=json.dumps({"prompt": f"tensor parallel request {i}", "max_tokens": 4,
                                                          "request_id": f"r{i}"}).encode(),
                                         headers={"Content-Type": "application/json"})
            out = json.loads(urllib.request.urlopen(req, timeout=60).read())
            assert out["request_id"] == f"r{i}" and out["ttft_ms"] > 0 and len(out["tokens"]) == 4
        procs[0].send_signal(signal.SIGTERM)
        for p in procs:
            assert p.wait(60) == 0
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
