"""Window timeline from a rocprofv3 CSV trace (``--kernel-trace --memory-copy-trace
--output-format csv``): per window, the big H2D's duration and period, the kernel-busy time
per period and how much of it overlaps the copy.

    python tools/timeline_csv.py gpurun_out/prof
"""

import argparse
import csv
import glob
import os
import statistics


def load(d):
    kt = glob.glob(os.path.join(d, "**", "*_kernel_trace.csv"), recursive=True)[0]
    mt = glob.glob(os.path.join(d, "**", "*_memory_copy_trace.csv"), recursive=True)[0]
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(kt))]
    ms = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r.get("Bytes", r.get("Size", 0)) or 0))
          for r in csv.DictReader(open(mt))]
    return sorted(ks), sorted(ms)


def union_len(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def clip(iv, a, b):
    return [(max(s, a), min(e, b)) for s, e in iv if e > a and s < b]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    a = ap.parse_args()
    ks, ms = load(a.dir)
    # the CSV copy trace has no byte counts: the window's event H2D is the long copy
    longest = max(m[1] - m[0] for m in ms)
    h2d = [m for m in ms if m[1] - m[0] > 0.5 * longest]
    kiv = [(s, e) for s, e, _ in ks]
    rows = []
    for j in range(1, len(h2d) - 1):
        s0, e0, _ = h2d[j]
        s1 = h2d[j + 1][0]
        rows.append(((s1 - s0) / 1e3, (e0 - s0) / 1e3, union_len(clip(kiv, s0, s1)) / 1e3,
                     union_len(clip(kiv, s0, e0)) / 1e3))
    med = lambda i: statistics.median(r[i] for r in rows)  # noqa: E731
    print(f"| quantity (median over {len(rows)} windows) | us |\n|---|---|")
    print(f"| window period (big H2D start to start) | {med(0):.1f} |")
    print(f"| event H2D copy duration | {med(1):.1f} |")
    print(f"| kernel-busy time per period | {med(2):.1f} |")
    print(f"| kernel-busy time during the copy | {med(3):.1f} |")


if __name__ == "__main__":
    main()
