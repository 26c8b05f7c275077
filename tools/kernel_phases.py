"""Per-window kernel time breakdown from a rocprofv3 ``--kernel-trace --output-format csv`` run.

Windows are delimited by the engine's one ``k_pack`` (multi-GPU) or ``k_window_end`` (one GPU)
dispatch per window (ops/csrc/engine.hip);
the dispatches of each window are grouped by kernel and launch shape (grid / workgroup), and the
table reports, per group, the median over the last ``--windows`` windows of its summed duration
per window and of its dispatch count -- the unprofiled (no PMC) device time each phase costs.

    python tools/kernel_phases.py gpurun_out/prof --windows 20 --title ...
"""

import argparse
import collections
import csv
import glob
import os
import statistics


def load(d):
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
                shape = f"{r.get('Grid_Size', r.get('Grid_Size_X', '?'))}/{r.get('Workgroup_Size', r.get('Workgroup_Size_X', '?'))}"
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, shape))
    rows.sort()
    return rows


def windows(rows, markers=("k_pack", "k_window_end")):
    out, cur = [], []
    for r in rows:
        cur.append(r)
        if any(m in r[2] for m in markers):
            out.append(cur)
            cur = []
    return out


def summarise(d, n_last, title, prefix="mislo::"):
    wins = windows(load(d))[-n_last:]
    per = collections.defaultdict(lambda: [[] for _ in wins])
    span = []
    for i, w in enumerate(wins):
        mine = [r for r in w if r[2].startswith(prefix)]
        if mine:
            span.append((max(r[1] for r in mine) - min(r[0] for r in mine)) / 1e3)
        for s, e, name, shape in mine:
            per[(name, shape)][i].append((e - s) / 1e3)
    rows = []
    for (name, shape), lists in per.items():
        tot = [sum(x) for x in lists]
        cnt = [len(x) for x in lists]
        rows.append((name, shape, statistics.median(cnt), statistics.median(tot)))
    rows.sort(key=lambda r: -r[3])
    total = sum(r[3] for r in rows)
    out = [f"# {title}", "", f"{len(wins)} windows (delimited by k_pack / k_window_end); median per window.", "",
           "| kernel | grid/wg | dispatches / window | us / window | share % |", "|---|---|---|---|---|"]
    for r in rows:
        out.append(f"| `{r[0]}` | {r[1]} | {r[2]:.0f} | {r[3]:.1f} | {100 * r[3] / total:.1f} |")
    out += ["", f"Sum of kernel time per window: **{total:.1f} us**; first-to-last mislo kernel span per window: "
                f"median {statistics.median(span):.1f} us." if span else ""]
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("dir")
    ap.add_argument("--windows", type=int, default=20)
    ap.add_argument("--title", default="per-window kernel time")
    ap.add_argument("--prefix", default="mislo::")
    a = ap.parse_args()
    print(summarise(a.dir, a.windows, a.title, a.prefix))


if __name__ == "__main__":
    main()
