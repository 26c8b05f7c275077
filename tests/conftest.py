import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

FIXTURES = os.path.join(ROOT, "tests", "fixtures")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP extension")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch

        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture
def fixtures_dir():
    return FIXTURES


class _Recorder:
    """Tiny local HTTP server (REF tests use httptest.NewServer): records requests and
    answers with a scripted sequence of (status, body) responses."""

    def __init__(self, responses=None):
        import http.server
        import threading

        self.requests = []
        self.responses = list(responses or [])
        rec = self

        class H(http.server.BaseHTTPRequestHandler):
            def _handle(self):
                n = int(self.headers.get("Content-Length") or 0)
                body = self.rfile.read(n) if n else b""
                rec.requests.append({"method": self.command, "path": self.path, "headers": dict(self.headers),
                                     "body": body})
                status, payload = rec.responses.pop(0) if rec.responses else (200, b"{}")
                if callable(payload):
                    payload = payload(self.path)
                if isinstance(payload, str):
                    payload = payload.encode()
                self.send_response(status)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(payload)))
                self.end_headers()
                self.wfile.write(payload)

            do_GET = do_POST = _handle

            def log_message(self, *a):
                pass

        self.httpd = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.url = f"http://127.0.0.1:{self.httpd.server_address[1]}"
        self.thread = threading.Thread(target=self.httpd.serve_forever, daemon=True)
        self.thread.start()

    def close(self):
        self.httpd.shutdown()
        self.httpd.server_close()


@pytest.fixture
def http_recorder():
    made = []

    def make(responses=None):
        r = _Recorder(responses)
        made.append(r)
        return r

    yield make
    for r in made:
        r.close()


# the agent CLI sets these for the HIP runtime it is about to start (cli/agent.py parse): a test
# that parses agent flags must not leave them to the tests after it in this process
_RUNTIME_ENV = ("GPU_MAX_HW_QUEUES", "MISLO_ONE_STREAM", "HSA_ENABLE_SDMA")


@pytest.fixture(autouse=True)
def _restore_runtime_env():
    saved = {k: os.environ.get(k) for k in _RUNTIME_ENV}
    yield
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
