#!/usr/bin/env bash
# usage: render_compatibility_report.sh [input-dir] [out-file]   (RUN_ID names the source run)
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
exec python3 "$ROOT/scripts/ci/kernel_compat.py" render --input-dir "${1:-artifacts/compatibility}" --out "${2:-docs/compatibility.md}"
