"""Built extensions load against the HIP runtime PyTorch ships: the agent engine shares that
runtime in-process (bench.py, smoke), so a HIP API newer than torch's libamdhip64 (e.g. a
hip_7.1-versioned symbol from /opt/rocm's headers) links here but fails to import on the box."""

import glob
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


def _versions(lib: str, defined: bool):
    out = subprocess.run(["objdump", "-T", lib], capture_output=True, text=True, check=True).stdout
    vs = set()
    for ln in out.splitlines():
        parts = ln.split()
        if len(parts) < 2 or "hip_" not in ln:
            continue
        is_und = "*UND*" in ln
        if is_und != (not defined):
            continue
        vs.update(p.strip("()") for p in parts if p.strip("()").startswith("hip_"))
    return vs


def test_extensions_need_only_torch_hip_symbol_versions():
    if shutil.which("objdump") is None:
        pytest.skip("needs objdump")
    torch = pytest.importorskip("torch")
    torch_hip = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
    if not os.path.exists(torch_hip):
        pytest.skip("torch without a bundled HIP runtime")
    have = _versions(torch_hip, defined=True)
    libs = glob.glob(os.path.join(ROOT, "llm_slo_ebpf_toolkit_amd", "**", "*.so"), recursive=True)
    assert libs, "run python -m llm_slo_ebpf_toolkit_amd.ops.build"
    for lib in libs:
        need = _versions(lib, defined=False)
        assert need <= have, (os.path.basename(lib), sorted(need - have))
