#!/usr/bin/env bash
# Ephemeral GitHub Actions runner loop for an MI355X host (REF infra/runner/aws: EC2 + cloud-init;
# MI355X nodes are bare metal or GPU VMs, so this is a systemd service instead of Terraform).
#
# Each iteration: GPU health gate -> fetch a registration token with the PAT -> configure an
# --ephemeral runner (labels self-hosted,linux,mi355x,gfx950,ebpf,kernel-X-Y) -> run exactly one
# job -> scrub the work directory and the toolkit's shared-memory rings -> repeat. A host whose
# GPUs fail the health gate stops taking jobs (runner-health.yml then reports it offline).
#
# Environment (from /etc/mislo-runner.env): GITHUB_REPOSITORY=owner/repo, RUNNER_PAT (repo
# admin:runner scope), RUNNER_DIR (actions-runner install), RUNNER_NAME_PREFIX (default: host name)
set -euo pipefail

: "${GITHUB_REPOSITORY:?set GITHUB_REPOSITORY}"
: "${RUNNER_PAT:?set RUNNER_PAT}"
RUNNER_DIR="${RUNNER_DIR:-/opt/actions-runner}"
PREFIX="${RUNNER_NAME_PREFIX:-$(hostname -s)}"
KVER="$(uname -r | awk -F. '{print "kernel-"$1"-"$2}')"
LABELS="self-hosted,linux,mi355x,gfx950,ebpf,${KVER}"
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"

gpu_healthy() {
  # gfx950 visible through KFD, every GPU answering rocm-smi, no pending RAS errors
  rocminfo 2>/dev/null | grep -q gfx950 || return 1
  rocm-smi --showuse >/dev/null 2>&1 || return 1
  if rocm-smi --showrasinfo all 2>/dev/null | grep -Eiq 'uncorrectable[^0-9]*[1-9]'; then return 1; fi
  return 0
}

scrub() {
  rm -rf "${RUNNER_DIR}/_work/"* 2>/dev/null || true
  rm -f /dev/shm/mislo-* 2>/dev/null || true   # rings a cancelled job left behind
}

while true; do
  if ! gpu_healthy; then
    echo "$(date -Is) GPU health gate failed; not taking jobs" >&2
    sleep 300
    continue
  fi
  token="$(curl -sf -X POST -H "Authorization: Bearer ${RUNNER_PAT}" -H "Accept: application/vnd.github+json" \
    "https://api.github.com/repos/${GITHUB_REPOSITORY}/actions/runners/registration-token" | jq -r .token)"
  if [[ -z "$token" || "$token" == "null" ]]; then
    echo "$(date -Is) could not obtain a registration token" >&2
    sleep 60
    continue
  fi
  name="${PREFIX}-$(date +%s)"
  (cd "$RUNNER_DIR" && ./config.sh --unattended --ephemeral --replace --name "$name" --labels "$LABELS" \
     --url "https://github.com/${GITHUB_REPOSITORY}" --token "$token" --work _work)
  (cd "$RUNNER_DIR" && ./run.sh) || echo "$(date -Is) runner exited with $?" >&2
  scrub
  "$HERE/preflight.sh" || true
done
