#!/usr/bin/env bash
# Post-job check on an MI355X runner: GPUs idle (no leftover processes holding /dev/kfd),
# HBM back to baseline, toolkit shared memory gone. Prints a one-line JSON status.
set -uo pipefail
busy="$(fuser /dev/kfd 2>/dev/null | wc -w)"
shm="$(ls /dev/shm 2>/dev/null | grep -c '^mislo-' || true)"
vram="$(rocm-smi --showmeminfo vram --json 2>/dev/null | jq '[.[] | .["VRAM Total Used Memory (B)"] | tonumber] | add // 0' 2>/dev/null || echo 0)"
printf '{"kfd_holders": %s, "mislo_shm": %s, "vram_used_bytes": %s}\n' "${busy:-0}" "${shm:-0}" "${vram:-0}"
[[ "${busy:-0}" -eq 0 && "${shm:-0}" -eq 0 ]]
