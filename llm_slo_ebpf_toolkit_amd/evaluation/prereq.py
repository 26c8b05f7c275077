"""Host prerequisite checks (`sloctl prereq check`), REF pkg/prereq/checker.go:22-251,
extended with the MI355X/ROCm prerequisites of the GPU path.

REF rows (same names, severities and remediation intent): host_linux, kernel_version
(>= 5.15), btf_available, kernel_headers, bpftool_installed, clang_installed,
privileged_execution, kind_installed, helm_installed. A report passes when every
*blocker* passes; ``strict_pass`` also requires the warnings.

Added rows (warnings, so a CPU-only replay host still passes; ``require_gpu`` promotes
them to blockers): rocm_installed (hipcc), amdgpu_kfd (/dev/kfd), gpu_gfx950 (an MI355X
agent visible to the ROCm runtime, read from the KFD topology -- no GPU context is
created), rccl_library, rocprofiler_sdk (the user-space GPU signal source).
"""

from __future__ import annotations

import glob
import json
import os
import platform
import re
import shutil
from dataclasses import asdict, dataclass, field
from typing import List, Optional, Tuple

from ..utils.timeutil import format_rfc3339_s, now_ns

BLOCKER = "blocker"
WARNING = "warning"
_KVER = re.compile(r"^(\d+)\.(\d+)")


@dataclass
class CheckResult:
    name: str
    pass_: bool
    severity: str
    current: str
    required: str
    remediation: str

    def to_dict(self):
        d = asdict(self)
        d["pass"] = d.pop("pass_")
        return {k: d[k] for k in ("name", "pass", "severity", "current", "required", "remediation")}


@dataclass
class Snapshot:
    host_os: str = ""
    host_arch: str = ""
    kernel_release: str = ""
    has_btf: bool = False
    has_kernel_hdrs: bool = False
    has_bpftool: bool = False
    has_clang: bool = False
    has_kind: bool = False
    has_helm: bool = False
    is_root: bool = False
    has_hipcc: bool = False
    has_kfd: bool = False
    gfx_targets: List[str] = field(default_factory=list)
    has_rccl: bool = False
    has_rocprofiler_sdk: bool = False


@dataclass
class Report:
    generated_at: str
    host_os: str
    host_arch: str
    kernel_release: str
    checks: List[CheckResult]
    pass_: bool

    def to_dict(self):
        return {"generated_at": self.generated_at, "host_os": self.host_os, "host_arch": self.host_arch,
                "kernel_release": self.kernel_release, "checks": [c.to_dict() for c in self.checks],
                "pass": self.pass_}


def parse_kernel_release(release: str) -> Tuple[int, int]:
    m = _KVER.match((release or "").strip())
    if not m:
        raise ValueError(f"unrecognized kernel release {release!r}")
    return int(m.group(1)), int(m.group(2))


def _rocm_root() -> str:
    return os.environ.get("ROCM_PATH", "/opt/rocm")


def kfd_gfx_targets(topology: str = "/sys/class/kfd/kfd/topology/nodes") -> List[str]:
    """gfx target names of GPU agents from the KFD topology (no HIP/HSA initialisation)."""
    out = []
    for props in sorted(glob.glob(os.path.join(topology, "*", "properties"))):
        try:
            with open(props) as fh:
                kv = dict(line.split(None, 1) for line in fh if " " in line.strip())
        except OSError:
            continue
        v = int(kv.get("gfx_target_version", "0").strip() or 0)
        if v:
            major, minor, step = v // 10000, (v // 100) % 100, v % 100
            out.append(f"gfx{major}{minor:x}{step:x}")
    return out


def collect_snapshot() -> Snapshot:
    rel = platform.release()
    rocm = _rocm_root()
    return Snapshot(
        host_os=platform.system().lower(), host_arch=platform.machine(), kernel_release=rel,
        has_btf=os.path.exists("/sys/kernel/btf/vmlinux"),
        has_kernel_hdrs=bool(rel) and os.path.exists(f"/lib/modules/{rel}/build"),
        has_bpftool=shutil.which("bpftool") is not None, has_clang=shutil.which("clang") is not None,
        has_kind=shutil.which("kind") is not None, has_helm=shutil.which("helm") is not None,
        is_root=(os.geteuid() == 0) if hasattr(os, "geteuid") else False,
        has_hipcc=os.path.exists(os.path.join(rocm, "bin", "hipcc")) or shutil.which("hipcc") is not None,
        has_kfd=os.path.exists("/dev/kfd"), gfx_targets=kfd_gfx_targets(),
        has_rccl=bool(glob.glob(os.path.join(rocm, "lib", "librccl.so*"))),
        has_rocprofiler_sdk=bool(glob.glob(os.path.join(rocm, "lib", "librocprofiler-sdk.so*"))),
    )


def _b(v: bool) -> str:
    return "true" if v else "false"


def _kernel_check(release: str) -> CheckResult:
    try:
        major, minor = parse_kernel_release(release)
    except ValueError:
        return CheckResult("kernel_version", False, BLOCKER, release, ">=5.15",
                           "Use Linux kernel 5.15+ for supported CO-RE signal set.")
    return CheckResult("kernel_version", major > 5 or (major == 5 and minor >= 15), BLOCKER, f"{major}.{minor}",
                       ">=5.15", "Upgrade Linux kernel to >=5.15 on validation hosts.")


def evaluate(s: Snapshot, require_gpu: bool = False) -> Report:
    gpu_sev = BLOCKER if require_gpu else WARNING
    checks = [
        CheckResult("host_linux", s.host_os == "linux", BLOCKER, s.host_os, "linux",
                    "Run prereq and privileged eBPF tests on a Linux host (self-hosted runner for CI)."),
        _kernel_check(s.kernel_release),
        CheckResult("btf_available", s.has_btf, BLOCKER, _b(s.has_btf), "true",
                    "Enable kernel BTF and ensure /sys/kernel/btf/vmlinux exists."),
        CheckResult("kernel_headers", s.has_kernel_hdrs, WARNING, _b(s.has_kernel_hdrs), "true",
                    "Install kernel headers matching uname -r for local probe build workflows."),
        CheckResult("bpftool_installed", s.has_bpftool, BLOCKER, _b(s.has_bpftool), "true",
                    "Install bpftool on Linux runner/host used for CO-RE generation and smoke tests."),
        CheckResult("clang_installed", s.has_clang, WARNING, _b(s.has_clang), "true",
                    "Install clang/llvm with the BPF target for probe object compilation."),
        CheckResult("privileged_execution", s.is_root, BLOCKER, _b(s.is_root), "true",
                    "Run in privileged context (root or CAP_BPF/CAP_PERFMON) for probe load tests."),
        CheckResult("kind_installed", s.has_kind, WARNING, _b(s.has_kind), "true",
                    "Install kind to run local multi-node integration lab."),
        CheckResult("helm_installed", s.has_helm, WARNING, _b(s.has_helm), "true",
                    "Install helm for optional chart-based deployment flows."),
        CheckResult("rocm_installed", s.has_hipcc, gpu_sev, _b(s.has_hipcc), "true",
                    "Install ROCm (hipcc) to build the gfx950 HIP kernels."),
        CheckResult("amdgpu_kfd", s.has_kfd, gpu_sev, _b(s.has_kfd), "true",
                    "Load the amdgpu driver and expose /dev/kfd and /dev/dri to the agent container."),
        CheckResult("gpu_gfx950", "gfx950" in s.gfx_targets, gpu_sev, ",".join(s.gfx_targets) or "none", "gfx950",
                    "Schedule the agent on MI355X nodes (gfx950) for the GPU attribution path."),
        CheckResult("rccl_library", s.has_rccl, gpu_sev, _b(s.has_rccl), "true",
                    "Install RCCL for the multi-GPU packet all-reduce over xGMI."),
        CheckResult("rocprofiler_sdk", s.has_rocprofiler_sdk, WARNING, _b(s.has_rocprofiler_sdk), "true",
                    "Install rocprofiler-sdk for the user-space GPU signal source (queue/HBM/xGMI/RCCL)."),
    ]
    ok = all(c.pass_ for c in checks if c.severity == BLOCKER)
    return Report(format_rfc3339_s(now_ns()), s.host_os, s.host_arch, s.kernel_release, checks, ok)


def run_local(require_gpu: bool = False) -> Report:
    return evaluate(collect_snapshot(), require_gpu)


def strict_pass(r: Report) -> bool:
    return all(c.pass_ for c in r.checks)


def to_json(r: Report) -> str:
    return json.dumps(r.to_dict(), indent=2)


def text_report(r: Report) -> str:
    nz = lambda v, f: v if v else f  # noqa: E731
    lines = [f"generated_at: {r.generated_at}", f"host: {r.host_os}/{r.host_arch}",
             f"kernel_release: {nz(r.kernel_release, 'unknown')}", "", "checks:"]
    for c in r.checks:
        lines.append(f"- [{'PASS' if c.pass_ else 'FAIL'}] ({c.severity.upper()}) {c.name}")
        lines.append(f"  current: {nz(c.current, 'n/a')}")
        lines.append(f"  required: {nz(c.required, 'n/a')}")
        lines.append(f"  remediation: {nz(c.remediation, 'n/a')}")
    lines.append("")
    lines.append("result: PASS (all blocker checks satisfied)" if r.pass_ else
                 "result: FAIL (one or more blocker checks failed)")
    return "\n".join(lines)

