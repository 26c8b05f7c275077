"""Workload-identity metadata and enrichers (the PID <-> cgroup <-> pod step).

REF pkg/signals/metadata.go:10-140: a static-defaults enricher chained after a
``/proc/<pid>/cgroup`` parser that derives the pod label (``pod<uid>`` path segment,
``.slice`` trimmed, ``_`` -> ``-``) and a 12-char container id (first segment with
>= 12 hex characters). NEW keeps an LRU cache per pid so the hot path does not
re-read procfs for every event, and exposes string interning used by the GPU records.
"""

from __future__ import annotations

import os
import threading
from collections import OrderedDict
from dataclasses import dataclass, replace
from typing import Dict, Optional, Tuple


@dataclass
class Metadata:
    node: str = ""
    namespace: str = ""
    pod: str = ""
    container: str = ""
    service: str = ""
    workload: str = ""
    pid: int = 0
    tid: int = 0
    trace_id: str = ""
    span_id: str = ""


def _fallback(v: str, d: str) -> str:
    return d if v == "" else v


class StaticMetadataEnricher:
    def __init__(self, defaults: Metadata):
        self.defaults = defaults

    def enrich(self, meta: Metadata) -> Metadata:
        d = self.defaults
        out = replace(meta)
        if not out.node:
            out.node = _fallback(d.node, "unknown-node")
        if not out.namespace:
            out.namespace = _fallback(d.namespace, "default")
        if not out.pod:
            out.pod = _fallback(d.pod, "unknown-pod")
        if not out.container:
            out.container = _fallback(d.container, "unknown-container")
        if not out.service:
            out.service = d.service
        if not out.workload:
            out.workload = d.workload
        if out.pid <= 0:
            out.pid = max(d.pid, os.getpid())
        if out.tid <= 0:
            out.tid = d.tid if d.tid > 0 else out.pid
        if not out.trace_id:
            out.trace_id = d.trace_id
        if not out.span_id:
            out.span_id = d.span_id
        return out


def _trim_set(s: str, chars: str) -> str:
    """Go strings.Trim(s, cutset): strip any chars of ``chars`` from both ends."""
    return s.strip(chars)


def normalize_pod_label(raw: str) -> str:
    if raw == "":
        return raw
    return _trim_set(raw, ".slice").replace("_", "-")


def likely_container_id(v: str) -> bool:
    if len(v) < 12:
        return False
    return sum(1 for ch in v if ("a" <= ch <= "f") or ("0" <= ch <= "9")) >= 12


def derive_from_cgroup_text(data: str) -> Tuple[str, str]:
    pod = container = ""
    for part in data.split("/"):
        p = part.strip()
        if not p:
            continue
        if not pod and p.startswith("pod"):
            pod = normalize_pod_label(p[3:])
            continue
        if not container and likely_container_id(p):
            container = p[:12]
    return pod, container


def derive_from_cgroup(pid: int, proc_root: str = "/proc") -> Tuple[str, str]:
    try:
        with open(f"{proc_root}/{pid}/cgroup", "r", encoding="utf-8", errors="replace") as fh:
            data = fh.read()
    except OSError:
        return "", ""
    return derive_from_cgroup_text(data)


class ProcMetadataEnricher:
    def __init__(self, nxt=None, proc_root: str = "/proc", cache_size: int = 4096):
        self.next = nxt
        self.proc_root = proc_root
        self._cache: "OrderedDict[int, Tuple[str, str]]" = OrderedDict()
        self._cache_size = cache_size
        self._lock = threading.Lock()

    def _lookup(self, pid: int) -> Tuple[str, str]:
        with self._lock:
            hit = self._cache.get(pid)
            if hit is not None:
                self._cache.move_to_end(pid)
                return hit
        res = derive_from_cgroup(pid, self.proc_root)
        with self._lock:
            self._cache[pid] = res
            if len(self._cache) > self._cache_size:
                self._cache.popitem(last=False)
        return res

    def enrich(self, meta: Metadata) -> Metadata:
        out = replace(meta)
        if out.pid > 0:
            pod, container = self._lookup(out.pid)
            if pod and not out.pod:
                out.pod = pod
                if not out.container:
                    out.container = container
        if self.next is not None:
            return self.next.enrich(out)
        return out


class Interner:
    """Dense string -> id interning (0 reserved for the empty string). Thread-safe."""

    def __init__(self, limit: int = 1 << 32):
        self._ids: Dict[str, int] = {"": 0}
        self._names = [""]
        self._limit = limit
        self._lock = threading.Lock()

    def id(self, name: str) -> int:
        i = self._ids.get(name)
        if i is not None:
            return i
        with self._lock:
            i = self._ids.get(name)
            if i is None:
                i = len(self._names)
                if i >= self._limit:
                    raise OverflowError("interner full")
                self._ids[name] = i
                self._names.append(name)
        return i

    def name(self, i: int) -> str:
        return self._names[i] if 0 <= i < len(self._names) else ""

    def names(self) -> list:
        """Every interned string in id order (id 0 = "")."""
        with self._lock:
            return list(self._names)

    def __len__(self) -> int:
        return len(self._names)
