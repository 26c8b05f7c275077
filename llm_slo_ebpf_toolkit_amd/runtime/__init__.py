"""Native host runtime: rings (in-process or shared memory, optionally pinned for DMA)
and paced replay producers, built in-tree by ``ops.build`` (``_mislo_rt`` pybind module and
``libmislo_rt.so`` with a C ABI for external producers)."""

from __future__ import annotations

import importlib
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libmislo_rt.so")


def load():
    try:
        return importlib.import_module(__name__ + "._mislo_rt")
    except ImportError as exc:
        raise RuntimeError("native runtime not built; run `python -m llm_slo_ebpf_toolkit_amd.ops.build`") from exc
