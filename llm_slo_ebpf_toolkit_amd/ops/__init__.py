"""Hand-written HIP/CDNA4 kernels for gfx950 and their bindings.

``load()`` imports the in-tree extension (``_mislo_hip``, built by ``ops.build``) and
uploads the signal-catalogue constant tables once per process. On a machine with a GPU
the extension is REQUIRED: a missing/stale build raises instead of silently falling back
to a CPU path (set ``MISLO_ALLOW_CPU_FALLBACK=1`` only for CPU-only development).
"""

from __future__ import annotations

import importlib
import os
import threading
from typing import Optional

import numpy as np

from ..signals import catalog

_LOCK = threading.Lock()
_MOD = None
_TABLES_SET = set()


class ExtensionMissing(RuntimeError):
    pass


def _import():
    try:
        return importlib.import_module(__name__ + "._mislo_hip")
    except ImportError as exc:  # pragma: no cover - exercised only without a build
        raise ExtensionMissing(
            "native extension _mislo_hip is not built; run `python -m llm_slo_ebpf_toolkit_amd.ops.build`"
        ) from exc


def tables_arrays():
    type_slot = np.full(128, -1, dtype=np.int8)
    for s in catalog.SIGNALS:
        type_slot[s.kernel_type] = s.slot
    scale = np.array([s.decode_scale for s in catalog.SIGNALS], dtype=np.float32)
    warn = np.array([s.warn for s in catalog.SIGNALS], dtype=np.float32)
    err = np.array([s.error for s in catalog.SIGNALS], dtype=np.float32)
    edges = np.array([list(s.buckets) + [float("inf")] * (16 - len(s.buckets)) for s in catalog.SIGNALS],
                     dtype=np.float32)
    assert edges.shape == (16, 16)
    return type_slot, scale, warn, err, edges


def load(device: Optional[int] = None):
    """Import the extension and upload the constant tables for ``device`` (current by default)."""
    global _MOD
    import torch

    with _LOCK:
        if _MOD is None:
            _MOD = _import()
        dev = torch.cuda.current_device() if device is None else int(device)
        if dev not in _TABLES_SET and torch.cuda.is_available():
            with torch.cuda.device(dev):
                _MOD.set_tables(*[torch.from_numpy(a) for a in tables_arrays()])
            _TABLES_SET.add(dev)
    return _MOD


_AGENT = None


def load_agent(init: bool = True):
    """The native window engine module (``_mislo_agent``: HIP + RCCL, no PyTorch) with the
    signal-catalogue constant tables uploaded. Raises ExtensionMissing without a build.
    ``init=False`` only imports it (no HIP call): for a process that still has to fork workers,
    which must happen before the HIP runtime initialises."""
    global _AGENT
    if not init:
        if _AGENT is not None:
            return _AGENT
        try:
            return importlib.import_module(__name__ + "._mislo_agent")
        except ImportError as exc:
            raise ExtensionMissing("native engine _mislo_agent is not built; run "
                                   "`python -m llm_slo_ebpf_toolkit_amd.ops.build`") from exc
    with _LOCK:
        if _AGENT is None:
            try:
                mod = importlib.import_module(__name__ + "._mislo_agent")
            except ImportError as exc:
                raise ExtensionMissing("native engine _mislo_agent is not built; run "
                                       "`python -m llm_slo_ebpf_toolkit_amd.ops.build`") from exc
            if mod.device_count() > 0:
                mod.set_tables(*tables_arrays())
            _AGENT = mod
    return _AGENT


def available() -> bool:
    try:
        _import()
        return True
    except ExtensionMissing:
        return False


def require_gpu_extension():
    """Fail loudly on a GPU machine without the native path."""
    import torch

    if torch.cuda.is_available() and not available() and os.environ.get("MISLO_ALLOW_CPU_FALLBACK") != "1":
        raise ExtensionMissing("GPU present but the HIP extension is not built")
