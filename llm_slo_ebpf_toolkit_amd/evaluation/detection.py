"""Detection delay measured on fault-onset episodes through the window engine.

REF reports a detection delay it never measures (a constant in its benchgen summary); round 2
here quoted ``window / 2 + attribution latency``. This module measures it: each episode is a
fault that starts at a uniformly random instant inside a collection window.

* the window holding the onset is the replay window with the faulted incident group's records
  *before* the onset drawn from the healthy profile (REF's base signal profile,
  pkg/signals/generator.go:244-259) and the fault's profile after it; the next window is faulted
  throughout (the replay holds a fault assignment for two windows);
* both windows go through the window engine (the CPU oracle engine here; the GPU engine is the
  same function of the same records, tests/test_native_engine.py), the first whose top-1 for the
  group is the injected domain detects it, and the attribution leaves when that window closes
  plus the engine's measured processing time for the window;
* delay = that emit time - onset. A fault undetected after both windows is a miss.

So the delay includes what the formula could not: how much of a window a fault must fill before
the evidence tips the posterior, and the windows in which it never does. Live runs measure the
same quantity from the agent's own output (tools/config2_evidence.py, tools/config3_evidence.py).
"""

from __future__ import annotations

import time
from typing import Dict, List

import numpy as np

from ..signals import catalog


def onset_episodes(n: int = 24, window_ms: int = 1000, seed: int = 7, model=None, scenario: str = "mixed",
                   events_per_window: int = 8192, spans_per_window: int = 512, services: int = 8) -> Dict[str, object]:
    from ..models.bayes import NaiveBayes
    from ..pipeline.cpu import CpuWindowEngine
    from ..pipeline.replay import ReplayConfig, ReplayGenerator, _profile

    model = model if model is not None else NaiveBayes.ref()
    gen = ReplayGenerator(ReplayConfig(scenario=scenario, events_per_window=events_per_window,
                                       spans_per_window=spans_per_window, n_services=services, window_ms=window_ms,
                                       fault_hold=2, p_fault=1.0, seed=seed))
    eng = CpuWindowEngine(model, window_ms=float(window_ms))
    rng = np.random.default_rng(seed)
    W = window_ms * 1_000_000
    healthy = [_profile(())]
    by_type = {s.kernel_type: s for s in catalog.SIGNALS}
    delays: List[float] = []
    windows_needed: List[int] = []
    proc_s: List[float] = []
    misses = 0
    for _ in range(n):
        w1, w2 = gen.next_window(), gen.next_window()
        faulty = [g for g in range(w1.n_groups) if w1.group_domains[g] != ["unknown"]]
        if not faulty:
            continue
        g = int(rng.choice(faulty))
        truth = set(w1.group_domains[g])
        u = float(rng.uniform(0.0, 1.0))
        onset = int(w1.t0_ns) + int(u * W)
        ev = w1.events.copy()
        pre = (ev["svc_id"].astype(np.int64) == g + 1) & (ev["ts_ns"].astype(np.int64) < onset)
        idx = np.flatnonzero(pre)
        names = np.array([by_type[int(t)].name if int(t) in by_type else "" for t in ev["signal_type"][idx]])
        ok = names != ""
        idx, names = idx[ok], names[ok]
        if len(idx):
            vals = gen._values(names, np.zeros(len(idx), dtype=np.int64), healthy)
            scale = np.array([catalog.BY_NAME[x].decode_scale for x in names])
            ev["value"][idx] = np.round(vals / scale).astype(np.uint64)
        detected = None
        for k, (events, spans) in enumerate(((ev, w1.spans), (w2.events, w2.spans))):
            t = time.perf_counter()
            r = eng.run(events, spans, w1.n_groups)
            proc_s.append(time.perf_counter() - t)
            top = catalog.ALL_DOMAINS[int(r.pred[g])]
            if top in truth:
                end = int(w1.t0_ns) + (k + 1) * W
                detected = (end - onset) / 1e9 + proc_s[-1]
                windows_needed.append(k + 1)
                break
        if detected is None:
            misses += 1
        else:
            delays.append(detected)
    d = np.array(delays) if delays else np.zeros(0)
    return {
        "episodes": len(delays) + misses, "detected": len(delays), "misses": misses,
        "detection_delay_seconds_median": float(np.median(d)) if len(d) else None,
        "detection_delay_seconds_p95": float(np.percentile(d, 95)) if len(d) else None,
        "detected_in_onset_window": int(sum(1 for k in windows_needed if k == 1)),
        "window_seconds": window_ms / 1000.0,
        "delays_seconds": [round(x, 4) for x in delays],
        "engine_seconds_per_window_median": float(np.median(proc_s)) if proc_s else None,
        "method": "fault onset uniform in a window; healthy records before it; first window whose top-1 "
                  "is the injected domain, emitted at the window's close + measured engine time",
    }

