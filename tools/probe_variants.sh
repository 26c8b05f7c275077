#!/usr/bin/env bash
# A/B builds of the window kernels: each variant is a self-contained copy of bench.py, the package
# and its fixtures under _variants/<name>/, with the native extensions rebuilt there with extra -D
# flags (join.hip: MISLO_PROBE_DEPTH, MISLO_PROBE_MINWG, ...). The shipped tree is untouched; the
# variants travel to the GPU box with the snapshot and run side by side in one session.
#
#   bash tools/probe_variants.sh build d2o3 "-DMISLO_PROBE_DEPTH=2 -DMISLO_PROBE_MINWG=3"   # here (CPU)
#   bash tools/probe_variants.sh bench d2o3 [bench.py args]                                    # on the box
#   bash tools/probe_variants.sh run prof tools/probe_profile.py --windows 4                    # on the box
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cmd=${1:?build|bench|clean}; name=${2:?variant name}; shift 2
V="$ROOT/_variants/$name"
case "$cmd" in
  build)
    defines=${1:-}
    rm -rf "$V" && mkdir -p "$V/tests/fixtures"
    cp "$ROOT/bench.py" "$V/" && mkdir -p "$V/tools" && cp "$ROOT/tools/probe_profile.py" "$V/tools/"
    cp -r "$ROOT/config" "$V/"
    cp "$ROOT/tests/fixtures/ref_multi_fault_samples.jsonl" "$V/tests/fixtures/"
    (cd "$ROOT" && tar --exclude='__pycache__' --exclude='_build' -cf - llm_slo_ebpf_toolkit_amd) | (cd "$V" && tar -xf -)
    if [ -n "${CSRC_REV:-}" ]; then  # the kernels of another commit (A/B against an earlier tree)
      for f in $(cd "$ROOT" && git ls-tree --name-only "$CSRC_REV" llm_slo_ebpf_toolkit_amd/ops/csrc/); do
        (cd "$ROOT" && git show "$CSRC_REV:$f") > "$V/$f"
      done
      defines="$defines (csrc from $CSRC_REV)"
    fi
    (cd "$V" && MISLO_HIP_DEFINES="${defines%% (csrc*}" python3 -m llm_slo_ebpf_toolkit_amd.ops.build --only agent --force)
    rm -rf "$V/llm_slo_ebpf_toolkit_amd/_build"
    echo "$defines" > "$V/DEFINES" ;;
  bench)
    cd "$V" && echo "variant $name: $(cat DEFINES)" && python3 -u bench.py "$@" ;;
  run)    # any script of the variant copy, e.g. tools/probe_profile.py
    cd "$V" && echo "variant $name: $(cat DEFINES)" && python3 -u "$@" ;;
  clean)
    rm -rf "$V" ;;
  *) echo "unknown command $cmd" >&2; exit 2 ;;
esac
