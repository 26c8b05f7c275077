"""How far the burn-rate forecast error can fall on the benchgen episodes.

Replays the episodes of ``evaluation/slo.py simulate_burn_prediction_error`` (the same draws in
the same order; checked against the simulator's own number) and scores other forecasts made at
the same windows against the same realised burns:

* ``segment``: the shipped forecaster (must equal the simulator's figure);
* ``persistence``: the round-5 forecaster;
* ``oracle``: the episode's true burn rate -- the floor set by the realised burn's own noise;
* ``known_plateau_start``: the mean burn since the fault's plateau began, the start given by the
  simulator -- the best a plateau-mean estimator can do, told what no window shows;
* ``ramp_ml``: a maximum-likelihood fit of the simulator's own shape (base rate, linear ramp of
  any start and length, plateau) to the last 80 windows, for the first 30 forecasts after
  detection (where the segment forecast is biased low by ramp windows), segment after that.

Usage: python tools/burn_floor.py [--samples tests/fixtures/ref_multi_fault_samples.jsonl]
Prints one JSON object (overall error and the error per 30-window band of forecast age)."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from llm_slo_ebpf_toolkit_amd.evaluation import slo  # noqa: E402
from llm_slo_ebpf_toolkit_amd.models import sample  # noqa: E402


def episodes(rates, seed=42, target=0.99, horizon=300, short=30, rpw=50.0):
    """The simulator's episodes, with both forecasters' per-window forecasts."""
    rng = np.random.default_rng(seed)
    budget = 1.0 - target
    out = []
    for i, b in enumerate(rates):
        b = float(b) if b and b > 0 else 2.0
        seg = slo.BurnRateForecaster(target, horizon, short)
        per = slo.BurnRateForecaster(target, horizon, short, method="persistence")
        p_base, p_fault = 0.1 * budget, min(1.0, b * budget)
        ramp = int(rng.integers(5, 31))
        lead = short + int(rng.integers(0, 60))
        det = None
        N, B, F, P = [], [], [], []
        for t in range(lead + ramp + 4 * horizon):
            x = min(1.0, max(0.0, (t - lead) / ramp))
            p = p_base + (p_fault - p_base) * x
            n = int(rng.poisson(rpw))
            br = int(rng.binomial(n, p)) if n else 0
            if det is None and t >= lead and seg.alert(i) > 1.0:
                det = t
            on = det is not None and t < det + horizon
            F.append(seg.observe(i, n, br, forecast=on))
            P.append(per.observe(i, n, br, forecast=on))
            N.append(n)
            B.append(br)
            if det is not None and t >= det + 2 * horizon:
                break
        out.append(dict(N=np.array(N, float), B=np.array(B, float), segment=np.array(F), persistence=np.array(P),
                        det=det, start=lead + ramp, burn=b, sim_err=seg.error()))
    return out


def score(eps, key, horizon=300, floor=0.05, budget=0.01):
    errs, age = [], np.zeros(horizon)
    for e in eps:
        if e["det"] is None:
            continue
        cn = np.concatenate([[0.0], np.cumsum(e["N"])])
        cb = np.concatenate([[0.0], np.cumsum(e["B"])])
        d, ee = e["det"], []
        for k in range(horizon):
            a, b = d + k + 1, d + k + 1 + horizon
            real = (cb[b] - cb[a]) / (cn[b] - cn[a]) / budget
            err = abs(e[key][d + k] - real) / max(real, floor)
            ee.append(err)
            age[k] += err
        errs.append(np.mean(ee))
    age /= len(errs)
    return float(np.mean(errs)), [round(float(age[a:a + 30].mean()), 4) for a in range(0, horizon, 30)]


def ramp_ml(N, B, t, budget=0.01, win=80):
    lo = max(0, t - win)
    n, b, tt = N[lo:t + 1], B[lo:t + 1], np.arange(lo, t + 1)
    pb = max(B[:lo + 1].sum(), 0.5) / max(N[:lo + 1].sum(), 1.0) if lo > 0 else 0.1 * budget
    Ls, Rs = np.arange(lo, t + 1), np.array([1, 3, 5, 8, 12, 16, 20, 25, 30, 40])
    X = np.clip((tt[None, None, :] - Ls[:, None, None]) / Rs[None, :, None], 0, 1).reshape(-1, len(tt))
    pf = np.full(X.shape[0], max(b.sum() / max(n.sum(), 1.0), 1.5 * pb))
    for _ in range(25):  # Newton on the plateau rate, every (start, length) at once
        Pm = np.clip(pb + (pf[:, None] - pb) * X, 1e-7, 1 - 1e-7)
        g = (X * (b / Pm - (n - b) / (1 - Pm))).sum(1)
        h = -(X * X * (b / Pm ** 2 + (n - b) / (1 - Pm) ** 2)).sum(1)
        pf = np.clip(pf - g / np.minimum(h, -1e-9), pb, 0.5)
    Pm = np.clip(pb + (pf[:, None] - pb) * X, 1e-7, 1 - 1e-7)
    ll = (b * np.log(Pm) + (n - b) * np.log1p(-Pm)).sum(1)
    return pf[int(np.argmax(ll))] / budget


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", default=os.path.join(ROOT, "tests", "fixtures", "ref_multi_fault_samples.jsonl"))
    ap.add_argument("--seed", type=int, default=42)
    a = ap.parse_args(argv)
    rates = [s.burn_rate for s in sample.load_samples_jsonl(a.samples)]
    eps = episodes(rates, a.seed)
    sim = slo.simulate_burn_prediction_error(rates, seed=a.seed)
    for e in eps:
        T = len(e["N"])
        e["oracle"] = np.full(T, e["burn"])
        cn = np.concatenate([[0.0], np.cumsum(e["N"])])
        cb = np.concatenate([[0.0], np.cumsum(e["B"])])
        lo = np.minimum(e["start"], np.arange(T))
        e["known_plateau_start"] = (cb[1:] - cb[lo]) / np.maximum(cn[1:] - cn[lo], 1.0) / 0.01
        e["ramp_ml"] = e["segment"].copy()
        if e["det"] is not None:
            for k in range(30):
                e["ramp_ml"][e["det"] + k] = ramp_ml(e["N"], e["B"], e["det"] + k)
    res = {"samples": len(rates), "simulator": sim}
    for key in ("segment", "persistence", "oracle", "known_plateau_start", "ramp_ml"):
        m, bands = score(eps, key)
        res[key] = {"error": round(m, 4), "error_by_age_band_30": bands}
    assert abs(res["segment"]["error"] - sim) < 1e-3, "replay diverged from the simulator"
    print(json.dumps(res))


if __name__ == "__main__":
    main()
