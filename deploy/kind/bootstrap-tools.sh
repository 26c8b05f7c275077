#!/usr/bin/env bash
# Check (and with AUTO_INSTALL=1, best-effort install) what the kind lab and the node build need:
# the cluster tools (docker, kubectl, kind, helm), the probe toolchain (clang with the bpf target,
# bpftool) and, on an MI355X node, the ROCm toolchain the agent's HIP engine is built with
# (hipcc with gfx950, rocprofv3) plus python3 with the agent's modules.
# Exit 0 when everything is present; 1 with the list of what is missing.
set -euo pipefail

AUTO_INSTALL="${AUTO_INSTALL:-0}"
OS="$(uname -s | tr '[:upper:]' '[:lower:]')"
ROCM="${ROCM_PATH:-/opt/rocm}"

missing=()
need() { command -v "$1" >/dev/null 2>&1 || missing+=("$1"); }
for bin in docker kubectl kind helm python3; do need "$bin"; done
if [[ "$OS" == "linux" ]]; then
  need bpftool
  if command -v clang >/dev/null 2>&1; then
    clang -print-targets 2>/dev/null | grep -q '\bbpf\b' || missing+=("clang(bpf target)")
  else
    missing+=("clang")
  fi
  # the GPU side: only where the node has AMD GPUs (KFD present)
  if [[ -e /dev/kfd || -d /sys/class/kfd ]]; then
    [[ -x "$ROCM/bin/hipcc" ]] || missing+=("hipcc(ROCm)")
    [[ -x "$ROCM/bin/rocprofv3" ]] || missing+=("rocprofv3(ROCm)")
    if [[ -x "$ROCM/bin/hipcc" ]] && ! "$ROCM/bin/hipcc" --offload-arch=gfx950 -x hip -c /dev/null -o /dev/null 2>/dev/null; then
      missing+=("hipcc gfx950 target")
    fi
  fi
fi
python3 - <<'PY' 2>/dev/null || missing+=("python3 modules (numpy, pyyaml, safetensors)")
import numpy, yaml, safetensors  # noqa: F401
PY

if [[ ${#missing[@]} -eq 0 ]]; then
  echo "all required tools are installed"
  exit 0
fi
echo "missing tools: ${missing[*]}"

if [[ "$AUTO_INSTALL" != "1" ]]; then
  echo
  echo "set AUTO_INSTALL=1 to run best-effort install commands; recommended manual installs:"
  if [[ "$OS" == "darwin" ]]; then
    echo "  brew install kubectl kind helm llvm"
  else
    echo "  sudo apt-get install -y bpftool clang llvm python3-numpy python3-yaml"
    echo "  ROCm (hipcc, rocprofv3): the AMD ROCm packages for your distribution (amdgpu-install)"
    echo "  kind / helm / kubectl: the vendors' release binaries"
  fi
  exit 1
fi

if [[ "$OS" == "darwin" ]]; then
  command -v brew >/dev/null 2>&1 || { echo "brew is required for AUTO_INSTALL on macOS" >&2; exit 1; }
  brew install kubectl kind helm llvm
  echo "macOS tool bootstrap complete"
  exit 0
fi
command -v apt-get >/dev/null 2>&1 || { echo "automatic Linux install supports apt-get only" >&2; exit 1; }
[[ "$(id -u)" -eq 0 ]] || { echo "run AUTO_INSTALL=1 as root for apt installs" >&2; exit 1; }
apt-get update
apt-get install -y bpftool clang llvm python3-numpy python3-yaml
for bin in kubectl helm kind; do
  command -v "$bin" >/dev/null 2>&1 || echo "install $bin from its vendor release (not in the distribution archive)"
done
if [[ -e /dev/kfd ]] && [[ ! -x "$ROCM/bin/hipcc" ]]; then
  echo "this node has AMD GPUs but no ROCm: install ROCm 7.x (amdgpu-install --usecase=rocm)"
fi
echo "linux tool bootstrap complete (see the notes above for tools outside apt)"
