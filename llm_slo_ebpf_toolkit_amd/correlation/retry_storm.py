"""Per-pod TCP-retransmit storm detection over a sliding window.

REF pkg/correlation/retry_storm.go:10-110 (window 10 s, threshold 5, prune strictly
older than ``now - window``). The batched GPU form is ``ops.storm.windowed_counts``
(segmented count over (pod, ts)-sorted keys); this class is the streaming CPU form the
agent uses per event and the oracle for the kernel.
"""

from __future__ import annotations

import threading
from collections import defaultdict
from typing import Dict, List

from ..utils.timeutil import SECOND

DEFAULT_STORM_WINDOW_NS = 10 * SECOND
DEFAULT_STORM_THRESHOLD = 5


class RetryStormDetector:
    def __init__(self, window_ns: int = DEFAULT_STORM_WINDOW_NS, threshold: int = DEFAULT_STORM_THRESHOLD):
        self.window_ns = window_ns
        self.threshold = threshold
        self._lock = threading.Lock()
        self._buckets: Dict[str, List[int]] = defaultdict(list)

    def _prune(self, events: List[int], now_ns: int) -> List[int]:
        # Events are kept in arrival order; REF drops the leading run of events strictly
        # before the cutoff (retry_storm.go:98-110), so out-of-order stragglers survive.
        cutoff = now_ns - self.window_ns
        i = 0
        while i < len(events) and events[i] < cutoff:
            i += 1
        return events[i:] if i else events

    def record(self, pod: str, ts_ns: int) -> bool:
        with self._lock:
            ev = self._buckets[pod]
            ev.append(ts_ns)
            ev = self._prune(ev, ts_ns)
            self._buckets[pod] = ev
            return len(ev) >= self.threshold

    def is_storm(self, pod: str, now_ns: int) -> bool:
        with self._lock:
            if pod not in self._buckets:
                return False
            ev = self._prune(self._buckets[pod], now_ns)
            self._buckets[pod] = ev
            return len(ev) >= self.threshold

    def count(self, pod: str, now_ns: int) -> int:
        with self._lock:
            if pod not in self._buckets:
                return 0
            ev = self._prune(self._buckets[pod], now_ns)
            self._buckets[pod] = ev
            return len(ev)

    def reset(self) -> None:
        with self._lock:
            self._buckets = defaultdict(list)
