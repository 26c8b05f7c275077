"""CPU model of the engine's per-window row protocol (ops/csrc/exchange.hip, engine.hip).

Per rank and window k, the device does:

1. part 1: decode the window's records (rows [0, counts[0])) into the current generation slot,
   and select this rank's trace-tagged local rows at warn level or above as 24-byte XRecs (time,
   trace hash, value, signal: no pod / pid / connection, so another GPU can only join them
   through the trace tier), capped at xchg_cap;
2. RCCL all-gather of every rank's fixed-size block [header: row count | XRecs] (comm stream);
3. part 2: decode the other ranks' rows after the window's own (capped at import_cap), partition
   the generation, and join this window's spans against every resident generation: the window's
   rows, and the rows of up to ``halo_windows`` earlier windows (their own records and the other
   ranks' rows they imported) that carry a signal and a timestamp with ts >= tmax_i - halo for
   every window i since theirs (tmax_i = window i's latest local record; a window without one
   ends the chain).

The join's row order -- which breaks ties between equally close candidates -- is [this window's
records | earlier windows' records, newest first | other ranks' rows, oldest window first], the
order nested per-window halo selections would produce. ``ExchangeModel`` runs exactly that over
the numpy oracle with a pluggable all-gather (a gloo process group in the tests, so the same
bytes cross a real process boundary), making the multi-GPU semantics testable on CPU; the GPU
test (test_native_engine) checks the device against the same oracle functions.
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
    w = XREC.itemsize
    cap = b.size // w - 1
    n = min(n, cap)
    rows = b[w:w + w * n].view(XREC)
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
    """One rank's window chain: resident generations (the halo) + other ranks' trace rows."""

    def __init__(self, rank: int, world: int, halo_ms: float, import_cap: int, xchg_cap: int,
                 allgather: Optional[Callable[[np.ndarray], List[np.ndarray]]] = None, halo_windows: int = 3):
        self.rank, self.world = rank, world
        self.halo_ns = int(round(halo_ms * 1e6))
        self.import_cap, self.xchg_cap = import_cap, xchg_cap
        self.halo_windows = halo_windows
        self.allgather = allgather
        self.gens: list = []                   # newest first: (local rows, other ranks' rows, tmax)
        self.injected = oracle.empty_rows()    # other ranks' rows for the next window (tests)
        self.sent = 0
        # rows lost to the capacities in the last window (the packet's dbg[5] / dbg[6])
        self.xchg_dropped = self.import_dropped = 0

    def block(self, d_loc: oracle.Decoded) -> Optional[np.ndarray]:
        """Part 1: this rank's exchange block for the window (what the GPU all-gathers)."""
        if self.world <= 1 or self.xchg_cap <= 0:
            return None
        mine = oracle.trace_rows(d_loc, len(d_loc.ts))
        self.sent = min(len(mine.ts), self.xchg_cap)
        self.xchg_dropped = len(mine.ts) - self.sent
        return oracle.exchange_blocks([mine], self.xchg_cap)

    def halo(self) -> oracle.Decoded:
        """The earlier generations' visible rows, in the join's row order (k_gen_begin cut-offs)."""
        if self.halo_ns <= 0:
            return oracle.empty_rows()
        locs, rems, cut = [], [], None
        for loc, rem, tmax in self.gens[:self.halo_windows]:
            if tmax == 0:
                break
            cut = tmax - self.halo_ns if cut is None else max(cut, tmax - self.halo_ns)
            locs.append(oracle.take(loc, (loc.slot != oracle.NO_SLOT) & (loc.ts != 0) & (loc.ts >= cut)))
            rems.append(oracle.take(rem, (rem.slot != oracle.NO_SLOT) & (rem.ts != 0) & (rem.ts >= cut)))
        out = oracle.empty_rows()
        for d in locs + rems[::-1]:
            out = oracle.concat(out, d)
        return out

    def join(self, d_loc: oracle.Decoded, spans: np.ndarray, n_groups: int, blocks=None, **join_kw):
        """Part 2: join [window rows | halo | other ranks' rows]; the window becomes a generation."""
        imp, self.injected = self.injected, oracle.empty_rows()
        for r, blk in enumerate(blocks or []):
            if r != self.rank:
                imp = oracle.concat(imp, parse_block(blk))
        self.import_dropped = max(0, len(imp.ts) - self.import_cap)
        imp = oracle.take(imp, np.arange(len(imp.ts)) < self.import_cap)
        d = oracle.concat(oracle.concat(d_loc, self.halo()), imp)
        res = oracle.join(d, spans, n_groups, **join_kw)
        res.n_rows = len(d.ts)
        self.gens = [(d_loc, imp, oracle.window_tmax(d_loc, len(d_loc.ts)))] + self.gens[:self.halo_windows - 1]
        return res

    def window(self, d_loc: oracle.Decoded, spans: np.ndarray, n_groups: int, **join_kw):
        self.xchg_dropped = self.import_dropped = 0
        blk = self.block(d_loc)
        blocks = self.allgather(blk) if blk is not None and self.allgather is not None else None
        return self.join(d_loc, spans, n_groups, blocks, **join_kw)
