"""Model images, record-level drivers and debug decoding around the window engine.

* ``GpuEngine`` -- a window of 64-byte EVENT / SPAN records (pipeline/replay.py, the incident
  lab) through the SHIPPED engine: the records go into page-locked user-space / span rings and
  the native ``WindowEngine`` (ops/csrc/engine.h, the agent's executor) DMAs, decodes, joins and
  scores them exactly as it does the agent's rings;
* ``KernelHarness`` -- the kernel unit-test harness (ops/csrc/bindings.cpp, a PyTorch extension):
  the same kernels launched one by one on torch tensors, with their intermediate buffers
  exposed (REF 40-byte record decode, EVENT16 wire decode, split chains, the refit kernel). It
  shares the engine's packet layout and packet kernels (mislo_packet.h); the agent, the
  benchmark and smoke() never use it.

Debug-counter decoding reproduces REF's DebugStats from the kernel's pair counts (join.hip).
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np

from ..collector import records
from ..models.bayes import MAX_PAIRS, N_DOMAINS, NOMINAL, LinearPosteriorModel
from ..signals import catalog
from . import load

N_DOMAINS_PAD = 16


def model_arrays_np(model: LinearPosteriorModel):
    """The PosteriorModel fields (numpy) of a host LinearPosteriorModel."""
    D = model.weights.shape[1]
    w = np.zeros((16, N_DOMAINS_PAD), dtype=np.float64)
    w[:, :D] = model.weights
    bias = np.full(N_DOMAINS_PAD, -np.inf, dtype=np.float64)
    bias[:D] = model.bias
    mean = model.mean if model.mean is not None else np.zeros(16)
    dom_mask = np.zeros(N_DOMAINS_PAD, dtype=np.int64)
    for d in range(D):
        dom_mask[d] = int(sum(1 << s for s in range(16) if model.evidence_mask[s, d]))
    table_mask = 0xFFFF if model.table_mask is None else int(sum(1 << s for s in range(16) if model.table_mask[s] > 0))
    mode = 0 if model.feature_mode == "binary" else 1
    return (w, bias, np.asarray(mean, dtype=np.float64), np.asarray(NOMINAL, dtype=np.float64),
            np.asarray(model.thresholds, dtype=np.float32), dom_mask, table_mask, mode)


MODEL_DTYPE = np.dtype([
    ("w", "<f8", (16, 16)), ("bias", "<f8", (16,)), ("mean", "<f8", (16,)), ("nominal", "<f8", (16,)),
    ("thr", "<f4", (16,)), ("dom_mask", "<u4", (16,)), ("table_mask", "<u4"), ("mode", "<i4"),
    ("n_pairs", "<i4"), ("_pad", "<i4"), ("pair_rho", "<f8"), ("w2", "<f8", (16, MAX_PAIRS)),
    ("bias2", "<f8", (MAX_PAIRS,)), ("pair_a", "u1", (MAX_PAIRS,)), ("pair_b", "u1", (MAX_PAIRS,)),
])
assert MODEL_DTYPE.itemsize == 9208  # == sizeof(mislo::PosteriorModel)


def model_bytes(model: LinearPosteriorModel) -> np.ndarray:
    """Byte image of ``mislo::PosteriorModel`` (ops/csrc/mislo_launch.h) for stream-ordered upload."""
    w, bias, mean, nominal, thr, dom_mask, table_mask, mode = model_arrays_np(model)
    rec = np.zeros(1, dtype=MODEL_DTYPE)
    rec["w"][0] = w
    rec["bias"][0] = bias
    rec["mean"][0] = mean
    rec["nominal"][0] = nominal
    rec["thr"][0] = thr
    rec["dom_mask"][0] = dom_mask.astype(np.uint32)
    rec["table_mask"][0] = table_mask
    rec["mode"][0] = mode
    rec["bias2"][0] = -np.inf
    if model.pairs is not None:
        P = len(model.pairs)
        rec["n_pairs"][0] = P
        rec["pair_rho"][0] = model.pair_rho
        rec["w2"][0][:, :P] = model.pair_w
        rec["bias2"][0][:P] = model.pair_b
        rec["pair_a"][0][:P] = model.pairs[:, 0]
        rec["pair_b"][0][:P] = model.pairs[:, 1]
    return rec.view(np.uint8)


APP_MODEL_DTYPE = np.dtype([
    ("w", "<f8", (16,)), ("b", "<f8", (16,)), ("w2", "<f8", (MAX_PAIRS,)), ("b2", "<f8", (MAX_PAIRS,)),
    ("thr_ms", "<f8"), ("dom_mask", "<u4"), ("on", "<i4"),
])
assert APP_MODEL_DTYPE.itemsize == 1040  # == sizeof(mislo::AppModel)


def app_model_bytes(model: LinearPosteriorModel) -> np.ndarray:
    """Byte image of ``mislo::AppModel`` (ops/csrc/mislo_launch.h): the model's application
    evidence (models/bayes.py AppEvidence) with the 2-fault columns of its pairs; ``on`` = 0
    without one."""
    rec = np.zeros(1, dtype=APP_MODEL_DTYPE)
    app = model.app
    if app is not None:
        D = model.weights.shape[1]
        w, b = app.terms()
        rec["w"][0][:D] = w[:D]
        rec["b"][0][:D] = b[:D]
        if model.pairs is not None:
            w2, b2 = app.pair_terms(model.pairs)
            rec["w2"][0][:len(w2)] = w2
            rec["b2"][0][:len(b2)] = b2
        rec["thr_ms"][0] = app.threshold_ms
        rec["dom_mask"][0] = int(sum(1 << d for d in range(D) if app.evidence_mask(D)[d]))
        rec["on"][0] = 1
    return rec.view(np.uint8)


def app_from_bytes(b: np.ndarray, n_dom: int = N_DOMAINS):
    """Inverse of ``app_model_bytes``: the AppEvidence an ``AppModel`` image evaluates, or None
    when the image is off."""
    from ..models.bayes import AppEvidence

    rec = np.frombuffer(np.ascontiguousarray(b, dtype=np.uint8).tobytes(), dtype=APP_MODEL_DTYPE)[0]
    if int(rec["on"]) == 0:
        return None
    return AppEvidence.from_image(np.array(rec["w"])[:n_dom], np.array(rec["b"])[:n_dom], np.array(rec["w2"]),
                                  np.array(rec["b2"]), float(rec["thr_ms"]), int(rec["dom_mask"]))


def model_from_bytes(b: np.ndarray) -> LinearPosteriorModel:
    """Inverse of ``model_bytes``: the host model a ``mislo::PosteriorModel`` image evaluates
    (the CPU window engine scores with it; exported model files hold the image)."""
    rec = np.frombuffer(np.ascontiguousarray(b, dtype=np.uint8).tobytes(), dtype=MODEL_DTYPE)[0]
    w = np.array(rec["w"], dtype=np.float64)
    bias = np.array(rec["bias"], dtype=np.float64)
    dom = np.array(rec["dom_mask"], dtype=np.uint32)
    D = N_DOMAINS
    mask = np.array([[(int(dom[d]) >> s) & 1 for d in range(D)] for s in range(16)], dtype=bool)
    tm = int(rec["table_mask"])
    mode = "binary" if int(rec["mode"]) == 0 else "continuous"
    mean = np.array(rec["mean"], dtype=np.float64) if mode == "continuous" else None
    table = np.array([(tm >> s) & 1 for s in range(16)], dtype=np.float64) if mode == "binary" else None
    m = LinearPosteriorModel("image", w[:, :D].copy(), bias[:D].copy(), mask, mode,
                             np.array(rec["thr"], dtype=np.float64), mean, table)
    P = int(rec["n_pairs"])
    if P:
        m.pair_w = np.array(rec["w2"], dtype=np.float64)[:, :P].copy()
        m.pair_b = np.array(rec["bias2"], dtype=np.float64)[:P].copy()
        m.pairs = np.stack([np.array(rec["pair_a"][:P]), np.array(rec["pair_b"][:P])], axis=1).astype(np.int64)
        m.pair_rho = float(rec["pair_rho"])
    return m


def decode_debug(dbg: np.ndarray, misc: np.ndarray, n_spans: int, n_events: int) -> Dict[str, int]:
    """Kernel pair counters -> REF DebugStats (correlator.go:20-25) + extras."""
    cand, low_raw, overlap, dropped, enriched = (int(x) for x in dbg[:5])
    unsupported_events = int(misc[0])
    low = low_raw - overlap
    n_sup = n_events - unsupported_events
    return {
        "candidates": cand, "low_confidence": low, "fanout_dropped": dropped,
        "unmatched": n_spans * n_sup - (cand + low), "unsupported_type": n_spans * unsupported_events,
        "spans_enriched": enriched,
    }


# device row records (ops/csrc/mislo_common.h SigRec / SpanRec), for inspection and tests
SIG_ROW = np.dtype([("ts", "<i8"), ("trace", "<u8"), ("conn", "<u8"), ("pod", "<u4"), ("pid", "<u4"),
                    ("svcnode", "<u4"), ("val", "<f4"), ("slot", "<u4"), ("pad", "V20")])
SPAN_ROW = np.dtype([("ts", "<i8"), ("trace", "<u8"), ("conn", "<u8"), ("pod", "<u4"), ("pid", "<u4"),
                     ("svcnode", "<u4"), ("group", "<u4"), ("pad", "V24")])
assert SIG_ROW.itemsize == 64 and SPAN_ROW.itemsize == 64


def signal_rows(eng, n: int) -> np.ndarray:
    """The first n decoded signal row records of an Engine (host copy)."""
    return eng.g_rec[: n * 64].cpu().numpy().view(SIG_ROW)


@dataclass
class WindowOutputs:
    hist: np.ndarray
    status: np.ndarray
    debug: Dict[str, int]
    feat: np.ndarray
    post: np.ndarray
    pred: np.ndarray
    conf: np.ndarray
    evbits: np.ndarray
    confusion: np.ndarray
    value_sum: np.ndarray  # [16] per-slot sums of decoded values (exact milli-unit integer sums)


class GpuEngine:
    """One window of 64-byte EVENT / SPAN records through the shipped WindowEngine."""

    def __init__(self, sig_cap: int, span_cap: int, group_cap: int, device: int = 0, window_ms: float = 2000.0,
                 threshold: float = 0.7, fanout: int = 3, group_mode: int = 1):
        from ..pipeline.window import RingWindowSource, WindowPipeline
        from ..runtime import load as load_rt

        rt = load_rt()
        pow2 = lambda n: 1 << max(4, int(np.ceil(np.log2(max(1, n)))))  # noqa: E731
        self.pipe = WindowPipeline(sig_cap, span_cap, group_cap, device, None, model="bayes", learn=False,
                                   window_ms=window_ms, threshold=threshold, fanout=fanout, group_mode=group_mode,
                                   user_cap=sig_cap, n_buffers=2, max_ahead=2)
        self.user, self.spans = rt.HostRing(pow2(2 * sig_cap), 64), rt.HostRing(pow2(2 * span_cap), 64)
        self.src = RingWindowSource(self.pipe, None, self.user, self.spans)
        self.sig_cap, self.span_cap, self.group_cap = sig_cap, span_cap, group_cap

    def set_model(self, model: LinearPosteriorModel) -> None:
        self.pipe.set_model(model)

    def process(self, events: np.ndarray, spans: np.ndarray, n_groups: int, labels=None,
                learn: bool = False) -> "WindowOutputs":
        from ..pipeline.window import Cut

        if events.dtype != records.EVENT or spans.dtype != records.SPAN:
            raise TypeError("events / spans must be 64-byte EVENT / SPAN records")
        if len(events) > self.sig_cap or len(spans) > self.span_cap or n_groups > self.group_cap:
            raise ValueError("window exceeds engine capacity")
        if len(events) and self.user.push(np.ascontiguousarray(events)) != len(events):
            raise RuntimeError("event ring full")
        if len(spans) and self.spans.push(np.ascontiguousarray(spans)) != len(spans):
            raise RuntimeError("span ring full")
        k = self.src.stage(Cut(kernel=0, user=self.user.head, spans=self.spans.head), n_groups, labels,
                           with_labels=labels is not None, learn=learn)["k"]
        pk = self.pipe.packet(k)
        r = self.pipe.results(k, n_groups)
        self.src.reap()
        return WindowOutputs(
            hist=pk["hist"].astype(np.int64), status=pk["status"].astype(np.int64),
            debug=decode_debug(pk["dbg"], pk["misc"], len(spans), len(events)), feat=r["feat"], post=r["post"],
            pred=r["pred"], conf=r["conf"], evbits=r["evbits"].view(np.uint32),
            confusion=pk["confusion"].astype(np.int64), value_sum=pk["misc"][2:18].astype(np.float64) * 1e-3)

    def close(self) -> None:
        self.src.drain()
        self.pipe.eng.close()


class KernelHarness:
    """Kernel unit-test harness over the PyTorch extension (see the module docstring)."""

    def __init__(self, sig_cap: int, span_cap: int, group_cap: int, device: int = 0, window_ms: float = 2000.0,
                 threshold: float = 0.7, fanout: int = 3, group_mode: int = 1):
        import torch

        self.torch = torch
        self.device = torch.device("cuda", device)
        self.mod = load(device)
        with torch.cuda.device(self.device):
            self.eng = self.mod.Engine(sig_cap, span_cap, group_cap, device)
            self.eng.set_join_params(window_ms, threshold, fanout, group_mode)
            self.ev_dev = torch.zeros(sig_cap * 64, dtype=torch.uint8, device=self.device)
            self.sp_dev = torch.zeros(span_cap * 64, dtype=torch.uint8, device=self.device)
            self.ev_host = torch.empty(sig_cap * 64, dtype=torch.uint8, pin_memory=True)
            self.sp_host = torch.empty(span_cap * 64, dtype=torch.uint8, pin_memory=True)
            self.cnt_host = torch.zeros(records.COUNTS_LEN, dtype=torch.int32, pin_memory=True)
            self.lab_host = torch.full((group_cap,), -1, dtype=torch.int32, pin_memory=True)
            self.copy_stream = torch.cuda.Stream(self.device)
        self.sig_cap, self.span_cap, self.group_cap = sig_cap, span_cap, group_cap
        self.n_events = self.n_spans = self.n_groups = 0
        self.wire, self.span_bytes = 64, 64
        self.ctx_dev = None

    # ---------------------------------------------------------------------------------
    def set_model(self, model: LinearPosteriorModel) -> None:
        with self.torch.cuda.device(self.device):
            self.eng.set_model_bytes(self.torch.from_numpy(model_bytes(model).copy()))

    def set_join_params(self, window_ms=2000.0, threshold=0.7, fanout=3, group_mode=1):
        self.eng.set_join_params(window_ms, threshold, fanout, group_mode)

    def set_ctx_rows(self, ids: np.ndarray, rows: np.ndarray) -> None:
        """Write context rows (id -> {pod, pid, conn32, svc<<16|node}) into the device context
        table the EVENT16 / SPAN20 decoders read (full 2^24-row id space, HBM-resident)."""
        torch = self.torch
        with torch.cuda.device(self.device):
            if self.ctx_dev is None:
                self.ctx_dev = torch.zeros((records.CTX_IDS, 4), dtype=torch.int32, device=self.device)
                self.eng.set_ctx_table(self.ctx_dev)
            if len(ids):
                idx = torch.from_numpy(np.asarray(ids, dtype=np.int64)).to(self.device)
                val = torch.from_numpy(np.ascontiguousarray(rows, dtype=np.uint32).view(np.int32).reshape(-1, 4))
                self.ctx_dev[idx] = val.to(self.device)
            torch.cuda.synchronize(self.device)

    def stage(self, events: np.ndarray, spans: np.ndarray, n_groups: int, labels: Optional[np.ndarray] = None,
              bases=None):
        """Copy records into pinned staging (host memcpy, no GPU work). ``events``: 64-byte EVENT
        or EVENT16 records (EVENT16 needs ``set_ctx_rows`` and the window's epoch ``bases``);
        ``spans``: 64-byte SPAN or SPAN20 records."""
        n, s = events.shape[0], spans.shape[0]
        if n > self.sig_cap or s > self.span_cap or n_groups > self.group_cap:
            raise ValueError("window exceeds engine capacity")
        if events.dtype not in records.WIRE_DTYPES.values() or spans.dtype not in (records.SPAN, records.SPAN20):
            raise TypeError("events/spans must use the EVENT|EVENT16 / SPAN|SPAN20 record dtypes")
        self.wire = records.wire_code(events.dtype)
        self.span_bytes = spans.dtype.itemsize
        self.ev_host.numpy()[: n * self.wire] = events.view(np.uint8).reshape(-1)
        self.sp_host.numpy()[: s * self.span_bytes] = spans.view(np.uint8).reshape(-1)
        c = self.cnt_host.numpy()
        c[:] = records.counts_row(n, s, n_groups, 0, bases if bases is not None else (0,), 0, self.span_bytes)
        lab = self.lab_host.numpy()
        lab[:] = -1
        if labels is not None:
            lab[: len(labels)] = labels
        self.n_events, self.n_spans, self.n_groups = n, s, n_groups

    def upload(self, stream=None) -> None:
        """Async H2D of the staged window on the copy stream; compute waits on an event."""
        torch = self.torch
        cs = self.copy_stream
        with torch.cuda.stream(cs):
            nb = self.n_events * self.wire
            self.ev_dev[:nb].copy_(self.ev_host[:nb], non_blocking=True)
            sb = self.n_spans * self.span_bytes
            self.sp_dev[:sb].copy_(self.sp_host[:sb], non_blocking=True)
            self.eng.counts.copy_(self.cnt_host, non_blocking=True)
            self.eng.labels.copy_(self.lab_host, non_blocking=True)
        (stream or torch.cuda.current_stream(self.device)).wait_stream(cs)

    def run(self, with_labels: bool = True, learn: bool = False) -> None:
        with self.torch.cuda.device(self.device):
            self.eng.run_window(self.ev_dev, self.sp_dev, self.n_groups, with_labels, learn, self.wire)

    def process(self, events, spans, n_groups, labels=None, learn=False) -> "WindowOutputs":
        self.stage(events, spans, n_groups, labels)
        self.upload()
        self.run(labels is not None, learn)
        return self.outputs()

    def outputs(self) -> WindowOutputs:
        e = self.eng
        self.torch.cuda.synchronize(self.device)
        G = self.n_groups
        dbg = e.dbg.cpu().numpy()
        misc = e.misc.cpu().numpy()
        return WindowOutputs(
            hist=e.hist.cpu().numpy().astype(np.int64), status=e.status_cnt.cpu().numpy().astype(np.int64),
            debug=decode_debug(dbg, misc, self.n_spans, self.n_events), feat=e.feat[:G].cpu().numpy(),
            post=e.post[:G].cpu().numpy(), pred=e.pred[:G].cpu().numpy(), conf=e.gconf[:G].cpu().numpy(),
            evbits=e.evbits[:G].cpu().numpy().view(np.uint32), confusion=e.confusion.cpu().numpy().astype(np.int64),
            value_sum=misc[2:18].astype(np.float64) * 1e-3)
