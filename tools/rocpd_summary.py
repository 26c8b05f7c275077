"""Summarise a rocprofv3 rocpd database (``<dir>/<name>_results.db``) into a markdown
kernel table for ``profiles/``: calls, total/avg/min/max us, share of GPU kernel time,
grid/workgroup shape, VGPR/AGPR/SGPR and LDS bytes (occupancy inputs)."""

import argparse
import sqlite3
import sys


def summarise(db: str, top: int = 25) -> str:
    c = sqlite3.connect(db)
    rows = list(c.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
        "max(grid_x), max(grid_y), max(workgroup_x), max(vgpr_count), max(accum_vgpr_count), max(sgpr_count), "
        "max(lds_size) from kernels group by name, grid_y order by sum(duration) desc"))
    total = sum(r[2] for r in rows) or 1.0
    unit = 1e-3  # rocpd durations are ns
    out = ["| kernel | calls | total us | avg us | min us | max us | % | grid | wg | vgpr | agpr | sgpr | lds B |",
           "|---|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows[:top]:
        name = r[0].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        out.append(f"| `{name}` | {r[1]} | {r[2] * unit:.1f} | {r[3] * unit:.2f} | {r[4] * unit:.2f} | "
                   f"{r[5] * unit:.2f} | {100 * r[2] / total:.1f} | {r[6]}x{r[7]} | {r[8]} | {r[9]} | {r[10]} | "
                   f"{r[11]} | {r[12]} |")
    out.append(f"\nTotal kernel time: {total * unit:.1f} us over {sum(r[1] for r in rows)} dispatches.")
    return "\n".join(out)


def timeline(db: str) -> str:
    """Window-period analysis: big host-to-device copies mark windows; for each period
    between consecutive big copies report copy time, kernel-busy time (union of kernel
    intervals) and how much of the copy overlapped kernels."""
    c = sqlite3.connect(db)
    try:
        big = c.execute("select max(size) from memory_copies").fetchone()[0] or 0
        min_copy = big // 2  # the event-array copy of each window
        copies = list(c.execute("select start, end, size from memory_copies where size >= ? order by start",
                                (min_copy,)))
    except sqlite3.Error:
        return "(no memory_copies table: run rocprofv3 with --memory-copy-trace)"
    kern = list(c.execute("select start, end from kernels order by start"))
    if len(copies) < 3:
        return f"(only {len(copies)} copies >= {min_copy} B)"

    def busy(a, b):  # union of kernel intervals clipped to [a, b)
        tot, cur_s, cur_e = 0, None, None
        for s, e in kern:
            if e <= a or s >= b:
                continue
            s, e = max(s, a), min(e, b)
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    tot += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            tot += cur_e - cur_s
        return tot

    rows = []
    for (s0, e0, n0), (s1, _, _) in zip(copies, copies[1:]):
        rows.append((s1 - s0, e0 - s0, busy(s0, s1), busy(s0, e0), n0))
    rows = rows[len(rows) // 4:]  # skip warm-up
    med = lambda xs: sorted(xs)[len(xs) // 2]
    us = 1e-3
    out = ["| quantity (median over windows) | us |", "|---|---|",
           f"| window period (big H2D start to start) | {med([r[0] for r in rows]) * us:.1f} |",
           f"| H2D copy duration ({rows[0][4] / 2**20:.1f} MiB) | {med([r[1] for r in rows]) * us:.1f} |",
           f"| kernel-busy time per period | {med([r[2] for r in rows]) * us:.1f} |",
           f"| kernel-busy time during the copy | {med([r[3] for r in rows]) * us:.1f} |",
           f"\n{len(rows)} windows analysed."]
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--title", default="")
    ap.add_argument("--timeline", action="store_true", help="also report the copy/compute window timeline")
    a = ap.parse_args()
    text = summarise(a.db, a.top)
    if a.timeline:
        text += "\n\n## Window timeline\n\n" + timeline(a.db)
    if a.title:
        text = f"# {a.title}\n\n" + text
    sys.stdout.write(text + "\n")


if __name__ == "__main__":
    main()
