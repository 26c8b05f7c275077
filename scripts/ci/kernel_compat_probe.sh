#!/usr/bin/env bash
# usage: kernel_compat_probe.sh --profile <label> --out <path>   (STRICT=true: fail on failed checks)
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
exec python3 "$ROOT/scripts/ci/kernel_compat.py" probe "$@"
