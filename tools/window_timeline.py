"""Window pipeline timeline from a rocprofv3 ``--kernel-trace --memory-copy-trace --output-format csv``
run of bench.py: where a window's period goes when the copy and the kernel chain each take less.

Windows are delimited by the engine's ``k_window_end`` / ``k_pack`` dispatch (ops/csrc/engine.hip).
For each of the last ``--windows`` windows it reports: the period (window end to window end), the
host-to-device copies attributed to the window (the H2D copies that end before its first kernel
and after the previous window's first kernel), the copy engine's busy and idle time within the
period, the kernel span (first start to last end), the time the window's first kernel waited after
its last copy ended, and the gap on the device between the previous window's last kernel and this
window's first one.

    python tools/window_timeline.py gpurun_out/r6_tl --windows 25
"""

import argparse
import csv
import glob
import json
import os
import statistics


def _rows(d, pattern):
    out = []
    for path in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        with open(path) as fh:
            out.extend(csv.DictReader(fh))
    return out


def load(d):
    ks = []
    for r in _rows(d, "*kernel_trace.csv"):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    ks.sort()
    cs = []
    for r in _rows(d, "*memory_copy_trace.csv"):
        direction = r.get("Direction", r.get("Kind", ""))
        if "HOST_TO_DEVICE" in direction.upper() or "H2D" in direction.upper():
            n = int(r.get("Bytes", r.get("Size", 0)) or 0)
            cs.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n))
    cs.sort()
    return ks, cs


def analyse(d, n_last):
    ks, cs = load(d)
    wins, cur = [], []
    for k in ks:
        if k[2].startswith("mislo::"):
            cur.append(k)
            if "k_window_end" in k[2] or "k_pack" in k[2]:
                wins.append(cur)
                cur = []
    wins = wins[-(n_last + 1):]
    rows = []
    for prev, w in zip(wins, wins[1:]):
        first, last = min(k[0] for k in w), max(k[1] for k in w)
        p_first, p_end = min(k[0] for k in prev), max(k[1] for k in prev)
        mine = [c for c in cs if p_first < c[1] <= first]
        period_lo = p_end
        busy = 0
        for s, e, _n in cs:
            lo, hi = max(s, period_lo), min(e, last)
            if hi > lo:
                busy += hi - lo
        rows.append({
            "period_us": (last - p_end) / 1e3,
            "kernel_span_us": (last - first) / 1e3,
            "device_gap_us": (first - p_end) / 1e3,
            "copies": len(mine),
            "copy_bytes": sum(c[2] for c in mine),
            "copy_span_us": (max(c[1] for c in mine) - min(c[0] for c in mine)) / 1e3 if mine else 0.0,
            "copy_sum_us": sum(c[1] - c[0] for c in mine) / 1e3,
            "first_kernel_after_last_copy_us": (first - max(c[1] for c in mine)) / 1e3 if mine else None,
            "copy_busy_in_period_us": busy / 1e3,
        })
    med = {k: statistics.median([r[k] for r in rows if r[k] is not None]) for k in rows[0]} if rows else {}
    return {"windows": len(rows), "median": med, "per_window": rows}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--windows", type=int, default=25)
    a = ap.parse_args(argv)
    print(json.dumps(analyse(a.dir, a.windows), indent=1))


if __name__ == "__main__":
    main()
