"""Nanosecond-exact time handling.

Correlation windows are compared with ``<=`` on nanosecond differences (REF
pkg/correlation/dns.go:107-113), so time is carried as int64 Unix nanoseconds
everywhere (Python ``datetime`` only has microseconds). ``0`` plays the role of Go's
zero ``time.Time`` (``IsZero``): a zero timestamp never matches any window.
"""

from __future__ import annotations

import calendar
import re
import time
from typing import Optional

ZERO = 0
NS = 1
US = 1_000
MS = 1_000_000
SECOND = 1_000_000_000
GO_ZERO_TIME = "0001-01-01T00:00:00Z"

_RE = re.compile(
    r"^(\d{4})-(\d{2})-(\d{2})[Tt ](\d{2}):(\d{2}):(\d{2})(?:\.(\d{1,9}))?([Zz]|[+-]\d{2}:\d{2})$"
)


def parse_rfc3339_ns(value: Optional[str]) -> int:
    """Parse an RFC3339(Nano) string to Unix ns. Empty/None/Go-zero -> 0."""
    if not value or value == GO_ZERO_TIME:
        return ZERO
    m = _RE.match(value.strip())
    if not m:
        raise ValueError(f"invalid RFC3339 timestamp {value!r}")
    y, mo, d, h, mi, s, frac, tz = m.groups()
    secs = calendar.timegm((int(y), int(mo), int(d), int(h), int(mi), int(s), 0, 0, 0))
    if tz not in ("Z", "z"):
        sign = 1 if tz[0] == "+" else -1
        secs -= sign * (int(tz[1:3]) * 3600 + int(tz[4:6]) * 60)
    ns = int((frac or "").ljust(9, "0")) if frac else 0
    return secs * SECOND + ns


def format_rfc3339_ns(ts_ns: int) -> str:
    """Format Unix ns like Go's time.Time MarshalJSON (RFC3339Nano, UTC, trailing zeros trimmed)."""
    if ts_ns == ZERO:
        return GO_ZERO_TIME
    secs, ns = divmod(int(ts_ns), SECOND)
    base = time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(secs))
    if ns:
        frac = f"{ns:09d}".rstrip("0")
        return f"{base}.{frac}Z"
    return base + "Z"


def format_rfc3339_s(ts_ns: int) -> str:
    """Second-precision RFC3339 (Go time.RFC3339 layout)."""
    secs = int(ts_ns) // SECOND
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(secs))


def now_ns() -> int:
    return time.time_ns()


def run_id(ts_ns: int) -> str:
    """REF benchmark run id layout 2006-01-02T15-04-05Z (pkg/benchmark/harness.go:88)."""
    return time.strftime("%Y-%m-%dT%H-%M-%SZ", time.gmtime(int(ts_ns) // SECOND))
