"""K5 release-gate statistics: GPU kernels (ops/csrc/gatestats.hip) + bit-identical numpy.

* ``bootstrap_quantiles`` -- [2, iters] q-quantiles of bootstrap resamples of the
  candidate and baseline samples. Resample index j of iteration it of set s is drawn from
  the counter-based stream ``splitmix64(ctr ^ splitmix64(seed))`` with
  ``ctr = s << 63 | it << 32 | j`` and mapped to [0, n) by Lemire's multiply-shift, so the
  numpy path (``*_np``) and the HIP kernel produce the same intervals bit for bit.
* ``rank_counts`` -- per element (all < v, all == v, y < v, y > v), from which the
  Mann-Whitney rank sum / tie correction and Cliff's delta follow without a sort.

REF counterparts: pkg/releasegate/gate.go:816-946 (mannWhitneyPValue, cliffsDelta,
bootstrapDeltaCI). REF's Go math/rand stream itself cannot be reproduced in Python.
"""

from __future__ import annotations

import math
from typing import Tuple

import numpy as np

from ..collector.records import splitmix64, splitmix64_np


def _indices_np(n: int, set_id: int, iters: int, seed: int) -> np.ndarray:
    seed_mix = np.uint64(splitmix64(int(seed) & ((1 << 64) - 1)))
    it = np.arange(iters, dtype=np.uint64)[:, None]
    j = np.arange(n, dtype=np.uint64)[None, :]
    ctr = (np.uint64(set_id) << np.uint64(63)) | (it << np.uint64(32)) | j
    x = splitmix64_np(ctr ^ seed_mix)
    with np.errstate(over="ignore"):
        return (((x >> np.uint64(32)) * np.uint64(n)) >> np.uint64(32)).astype(np.int64)


def _quantile_rows(s: np.ndarray, q: float) -> np.ndarray:
    n = s.shape[1]
    if n == 1:
        return s[:, 0].copy()
    pos = q * (n - 1)
    lo, hi = math.floor(pos), math.ceil(pos)
    if lo == hi:
        return s[:, lo].copy()
    f = pos - lo
    return s[:, lo] * (1 - f) + s[:, hi] * f


def bootstrap_quantiles_np(cand: np.ndarray, base: np.ndarray, q: float, iters: int, seed: int) -> np.ndarray:
    out = np.empty((2, iters), dtype=np.float64)
    for set_id, v in enumerate((cand, base)):
        sv = np.sort(np.asarray(v, dtype=np.float64))
        idx = _indices_np(len(sv), set_id, iters, seed)
        out[set_id] = _quantile_rows(sv[np.sort(idx, axis=1)], q)
    return out


def _signed64(seed: int) -> int:
    s = int(seed) & ((1 << 64) - 1)
    return s - (1 << 64) if s >= (1 << 63) else s


def bootstrap_quantiles(cand: np.ndarray, base: np.ndarray, q: float, iters: int, seed: int,
                        device: int = 0) -> np.ndarray:
    import torch

    from . import load

    mod = load(device)
    n_max = int(mod.BOOT_MAX_N)
    if len(cand) > n_max or len(base) > n_max:
        return bootstrap_quantiles_np(cand, base, q, iters, seed)
    dev = torch.device("cuda", device)
    c = torch.from_numpy(np.sort(np.asarray(cand, dtype=np.float64))).to(dev)
    b = torch.from_numpy(np.sort(np.asarray(base, dtype=np.float64))).to(dev)
    with torch.cuda.device(dev):
        out = mod.boot_quantile(c, b, float(q), int(iters), _signed64(seed))
    return out.cpu().numpy()


def bootstrap_quantile_delta(cand, base, q: float, iters: int, seed: int, use_gpu: bool = True) -> np.ndarray:
    qs = bootstrap_quantiles(cand, base, q, iters, seed) if use_gpu else \
        bootstrap_quantiles_np(np.asarray(cand), np.asarray(base), q, iters, seed)
    return qs[0] - qs[1]


def rank_counts_np(x: np.ndarray, y: np.ndarray) -> np.ndarray:
    v = np.concatenate([np.asarray(x, dtype=np.float64), np.asarray(y, dtype=np.float64)])
    ys = np.sort(np.asarray(y, dtype=np.float64))
    s = np.sort(v)
    lt_all = np.searchsorted(s, v, side="left")
    eq_all = np.searchsorted(s, v, side="right") - lt_all
    lt_y = np.searchsorted(ys, v, side="left")
    gt_y = len(ys) - np.searchsorted(ys, v, side="right")
    return np.stack([lt_all, eq_all, lt_y, gt_y]).astype(np.int64)


def rank_counts(x, y, device: int = 0) -> np.ndarray:
    import torch

    from . import load

    mod = load(device)
    v = np.concatenate([np.asarray(x, dtype=np.float64), np.asarray(y, dtype=np.float64)])
    t = torch.from_numpy(v).to(torch.device("cuda", device))
    with torch.cuda.device(device):
        out = mod.rank_counts(t, len(x))
    return out.cpu().numpy().view(np.uint32).astype(np.int64)


def stats_from_rank_counts(rc: np.ndarray, nx: int, ny: int) -> Tuple[float, float, float]:
    """(Mann-Whitney two-sided p with tie + continuity correction, Cliff's delta, U)."""
    lt_all, eq_all, lt_y, gt_y = (rc[k].astype(np.float64) for k in range(4))
    if nx == 0 or ny == 0:
        return 1.0, 0.0, 0.0
    ranks = lt_all + (eq_all + 1.0) / 2.0
    rank_x = float(ranks[:nx].sum())
    tie_sum = float((eq_all * eq_all - 1.0).sum())
    nxf, nyf = float(nx), float(ny)
    u1 = rank_x - nxf * (nxf + 1) / 2.0
    u = min(u1, nxf * nyf - u1)
    N = nxf + nyf
    var_u = (nxf * nyf / 12.0) * ((N + 1.0) - tie_sum / (N * (N - 1.0)))
    delta = float(lt_y[:nx].sum() - gt_y[:nx].sum()) / (nxf * nyf)
    if var_u <= 0:
        return 1.0, delta, u
    z = u - nxf * nyf / 2.0
    z = (z - 0.5) / math.sqrt(var_u) if z > 0 else (z + 0.5) / math.sqrt(var_u)
    p = 2 * (1 - 0.5 * (1 + math.erf(abs(z) / math.sqrt(2))))
    return min(max(p, 0.0), 1.0), delta, u
