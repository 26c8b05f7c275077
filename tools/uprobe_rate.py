"""How often would the agent's HIP / ROCr uprobes fire in an LLM workload? (ADVICE r5 low:
the workload-side cost of the uprobes on hsa_signal_wait_scacquire / _relaxed and hipMemcpy*.)

Uprobes need root, which the GPU boxes of this pool do not grant, so the cost is not measured by
attaching them. Instead this runs the demo's Llama decode loop (the config-3 backend: 1B, greedy,
one request at a time) for ``--seconds`` under ``rocprofv3 --hip-trace --hsa-trace --stats``;
the API statistics count every call the probes would trap on. The per-hit cost of a uprobe +
uretprobe pair (a breakpoint trap and a return trampoline, ~1-3 us on x86-64) times the calls per
second bounds the slowdown of the probed process:

    cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \\
      rocprofv3 --hip-trace --hsa-trace --stats --output-format csv -d gpurun_out/uprobe_rate -- \\
      python tools/uprobe_rate.py --seconds 10
    python tools/uprobe_rate.py --summarize gpurun_out/uprobe_rate
"""

from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PROBED = ("hsa_signal_wait_scacquire", "hsa_signal_wait_relaxed", "hipMemcpy", "hipMemcpyAsync",
          "hipStreamSynchronize", "hipDeviceSynchronize", "hipLaunchKernel")


def run(seconds: float, preset: str, max_tokens: int) -> dict:
    import torch

    from llm_slo_ebpf_toolkit_amd.models.llama import build

    model = build(preset, "cuda")
    x = torch.tensor([[1, 2, 3, 4, 5, 6, 7, 8]], device="cuda")
    model.generate(x, 2)
    t0, reqs, toks = time.time(), 0, 0
    while time.time() - t0 < seconds:
        r = model.generate(x, max_tokens)
        reqs += 1
        toks += int(r["new_tokens"])
    dt = time.time() - t0
    out = {"seconds": round(dt, 3), "requests": reqs, "tokens": toks, "tokens_per_s": round(toks / dt, 1)}
    print(json.dumps(out), flush=True)
    return out


def summarize(d: str) -> dict:
    calls = {}
    for path in glob.glob(os.path.join(d, "**", "*api_stats.csv"), recursive=True) + \
            glob.glob(os.path.join(d, "**", "*hsa_stats.csv"), recursive=True) + \
            glob.glob(os.path.join(d, "**", "*hip_stats.csv"), recursive=True):
        with open(path) as fh:
            for r in csv.DictReader(fh):
                name = r.get("Name") or r.get("FUNCTION") or ""
                try:
                    calls[name] = calls.get(name, 0) + int(float(r.get("Calls") or r.get("CALLS") or 0))
                except ValueError:
                    pass
    return {k: v for k, v in sorted(calls.items()) if any(k.startswith(p) for p in PROBED)}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--preset", default="1b")
    ap.add_argument("--max-tokens", type=int, default=8)
    ap.add_argument("--summarize", default="", help="a rocprofv3 output directory: the probed calls")
    ap.add_argument("--run-json", default="", help="the run's JSON line (tokens, seconds) for --summarize")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    if not a.summarize:
        run(a.seconds, a.preset, a.max_tokens)
        return 0
    calls = summarize(a.summarize)
    out = {"calls": calls}
    if a.run_json and os.path.exists(a.run_json):
        with open(a.run_json) as fh:
            line = [ln for ln in fh if ln.startswith("{")][-1]
        r = json.loads(line)
        out["run"] = r
        sec = max(r["seconds"], 1e-9)
        waits = sum(v for k, v in calls.items() if k.startswith("hsa_signal_wait") or k.startswith("hipMemcpy")
                    or k.endswith("Synchronize"))
        launches = sum(v for k, v in calls.items() if "Launch" in k)
        # a uprobe (+ uretprobe for the waits) per call, 1-3 us per hit (trap + return trampoline)
        for name, n in (("waits_copies_syncs", waits), ("launches", launches)):
            per_s = n / sec
            out[f"{name}_per_s"] = round(per_s, 1)
            out[f"{name}_pct_of_one_core_at_1us"] = round(per_s * 1e-6 * 100, 3)
            out[f"{name}_pct_of_one_core_at_3us"] = round(per_s * 3e-6 * 100, 3)
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(s)
    return 0


if __name__ == "__main__":
    sys.exit(main())
