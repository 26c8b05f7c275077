"""CPU model of the engine's per-window import protocol (ops/csrc/exchange.hip, engine.hip).

Per rank and window k, the device does:

1. part 1: decode the window's records plus the halo it imported from window k-1 (rows
   [counts[0], rows[0]): joined, never counted), and select this rank's trace-tagged local rows
   at warn level or above as 32-byte XRecs (time, trace hash, value, signal: no pod / pid /
   connection, so another GPU can only join them through the trace tier), capped at xchg_cap;
2. RCCL all-gather of every rank's fixed-size block [header: row count | XRecs] (comm stream);
3. part 2: decode the other ranks' rows (rows [rows[0], rows[1])), join everything, and select
   the next window's halo: rows (all of them) with a signal, a timestamp and
   ts >= tmax - halo, tmax = the window's latest local record, in row order, capped at
   import_cap; the next window's other-GPU rows are appended after it up to the same cap.

``ExchangeModel`` runs exactly that over the numpy oracle with a pluggable all-gather (a gloo
process group in the tests, so the same bytes cross a real process boundary), making the
multi-GPU semantics testable on CPU; the GPU test (test_native_engine) checks the device's
selections and merge against the same oracle functions.
"""

from __future__ import annotations

from typing import Callable, List, Optional

import numpy as np

from ..pipeline import oracle

XREC = oracle.XREC


def parse_block(block: np.ndarray) -> oracle.Decoded:
    """One rank's exchange block -> imported rows (oracle.remote_rows of its XRecs)."""
    b = np.ascontiguousarray(block, dtype=np.uint8)
    n = int(b[:4].view(np.uint32)[0])
    cap = b.size // 32 - 1
    n = min(n, cap)
    rows = b[32:32 + 32 * n].view(XREC)
    slot = np.where(rows["slot"] == 0xFF, oracle.NO_SLOT, rows["slot"]).astype(np.uint8)
    d = oracle.Decoded(rows["ts"].astype(np.int64), rows["val"].astype(np.float32), slot,
                       np.zeros(n, np.uint8), np.zeros(n, np.uint32), np.zeros(n, np.uint32), np.zeros(n, np.uint32),
                       rows["tr"].astype(np.uint64), np.zeros(n, np.uint64))
    return oracle.remote_rows(d)


def torch_allgather(group=None) -> Callable[[np.ndarray], List[np.ndarray]]:
    """All-gather of equal-size uint8 blocks over a torch.distributed group (gloo on CPU)."""

    def gather(block: np.ndarray) -> List[np.ndarray]:
        import torch
        import torch.distributed as dist

        t = torch.from_numpy(np.ascontiguousarray(block, dtype=np.uint8).copy())
        outs = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
        dist.all_gather(outs, t, group=group)
        return [o.numpy() for o in outs]

    return gather


class ExchangeModel:
    """One rank's window chain with imports (halo + other ranks' trace rows)."""

    def __init__(self, rank: int, world: int, halo_ms: float, import_cap: int, xchg_cap: int,
                 allgather: Optional[Callable[[np.ndarray], List[np.ndarray]]] = None):
        self.rank, self.world = rank, world
        self.halo_ns = int(round(halo_ms * 1e6))
        self.import_cap, self.xchg_cap = import_cap, xchg_cap
        self.allgather = allgather
        self.imports = oracle.empty_rows()
        self.sent = 0

    def block(self, d_loc: oracle.Decoded) -> Optional[np.ndarray]:
        """Part 1: this rank's exchange block for the window (what the GPU all-gathers)."""
        if self.world <= 1 or self.xchg_cap <= 0:
            return None
        mine = oracle.trace_rows(d_loc, len(d_loc.ts))
        self.sent = min(len(mine.ts), self.xchg_cap)
        return oracle.exchange_blocks([mine], self.xchg_cap)

    def join(self, d_loc: oracle.Decoded, spans: np.ndarray, n_groups: int, blocks=None, **join_kw):
        """Part 2: join [window rows | halo of k-1 | other ranks' rows], keep the next halo."""
        imp = self.imports
        for r, blk in enumerate(blocks or []):
            if r != self.rank:
                imp = oracle.concat(imp, parse_block(blk))
        imp = oracle.take(imp, np.arange(len(imp.ts)) < self.import_cap)
        d = oracle.concat(d_loc, imp)
        res = oracle.join(d, spans, n_groups, **join_kw)
        res.n_rows = len(d.ts)
        halo = oracle.halo_rows(d, len(d_loc.ts), self.halo_ns) if self.halo_ns > 0 else oracle.empty_rows()
        self.imports = oracle.take(halo, np.arange(len(halo.ts)) < self.import_cap)
        return res

    def window(self, d_loc: oracle.Decoded, spans: np.ndarray, n_groups: int, **join_kw):
        blk = self.block(d_loc)
        blocks = self.allgather(blk) if blk is not None and self.allgather is not None else None
        return self.join(d_loc, spans, n_groups, blocks, **join_kw)
