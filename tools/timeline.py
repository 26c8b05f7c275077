"""Where a window's period goes: the compute queue's idle gaps and what they wait for, from one
rocprofv3 ``--kernel-trace --memory-copy-trace --output-format csv`` run.

The engine overlaps window k+1's host-to-device copies with window k's kernel chain (three
buffers, ops/csrc/engine.hip). When the period exceeds both the chain and the copies, the
difference is time in which the compute queue is idle. Each idle gap between two windows' chains
is classified by what was running during it:
* copy: a host-to-device copy was in flight (the next chain waits for its window's bytes);
* host: nothing was in flight on the GPU (the next window had not been issued yet: host side).

    python tools/timeline.py gpurun_out/trace --windows 20 --title ...
"""

import argparse
import csv
import glob
import os
import statistics


def _rows(d, pattern):
    for path in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        with open(path) as fh:
            yield from csv.DictReader(fh)


def load(d, prefix="mislo::"):
    kern = []
    for r in _rows(d, "*kernel_trace.csv"):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        if name.startswith(prefix):
            kern.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    copies = []
    for r in _rows(d, "*memory_copy_trace.csv"):
        kind = (r.get("Direction") or r.get("Kind") or r.get("Operation") or "").upper()
        if "DEVICE_TO_HOST" in kind or "D2H" in kind:
            continue
        copies.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    kern.sort()
    copies.sort()
    return kern, copies


def union_len(iv, lo, hi):
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        s, e = max(s, lo), min(e, hi)
        if e <= s:
            continue
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def analyse(d, n_last, markers=("k_pack", "k_window_end"), first=("k_window_begin",)):
    kern, copies = load(d)
    wins, cur = [], []
    for r in kern:
        cur.append(r)
        if any(m in r[2] for m in markers):
            wins.append(cur)
            cur = []
    wins = wins[-(n_last + 1):]
    out = []
    for a, b in zip(wins, wins[1:]):
        end_a = max(r[1] for r in a)
        start_b = min(r[0] for r in b)
        end_b = max(r[1] for r in b)
        period = end_b - end_a
        chain = union_len([(s, e) for s, e, _ in b], start_b, end_b)
        gap = max(0, start_b - end_a)
        gap_copy = union_len(copies, end_a, start_b) if gap else 0
        inner_idle = (end_b - start_b) - chain  # idle inside the chain (dependencies, launch gaps)
        out.append({"period": period, "chain_busy": chain, "gap": gap, "gap_copy": gap_copy,
                    "gap_host": gap - gap_copy, "inner_idle": inner_idle,
                    "copy_busy": union_len(copies, end_a, end_b)})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--windows", type=int, default=20)
    ap.add_argument("--title", default="Window timeline")
    a = ap.parse_args()
    res = analyse(a.dir, a.windows)
    if not res:
        raise SystemExit("no windows found")
    med = {k: statistics.median(r[k] for r in res) / 1e3 for k in res[0]}
    lines = [f"# {a.title}", "", f"{len(res)} windows, median per window (us), window k = from the end of chain k-1 "
             "to the end of chain k.", "", "| | us |", "|---|---|"]
    for k, label in (("period", "period (chain end to chain end)"), ("chain_busy", "kernels busy"),
                     ("inner_idle", "idle inside the chain (launch / dependency gaps)"),
                     ("gap", "idle between chains"), ("gap_copy", "  of which a copy was in flight"),
                     ("gap_host", "  of which nothing was in flight (host)"), ("copy_busy", "copy engine busy")):
        lines.append(f"| {label} | {med[k]:.1f} |")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
