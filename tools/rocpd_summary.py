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
        "max(lds_size) from kernels group by name order by sum(duration) desc"))
    total = sum(r[2] for r in rows) or 1.0
    unit = 1e-3  # rocpd durations are ns
    out = ["| kernel | calls | total us | avg us | min us | max us | % | grid | wg | vgpr | agpr | sgpr | lds B |",
           "|---|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows[:top]:
        name = r[0].split("(")[0].replace("void ", "")
        out.append(f"| `{name}` | {r[1]} | {r[2] * unit:.1f} | {r[3] * unit:.2f} | {r[4] * unit:.2f} | "
                   f"{r[5] * unit:.2f} | {100 * r[2] / total:.1f} | {r[6]}x{r[7]} | {r[8]} | {r[9]} | {r[10]} | "
                   f"{r[11]} | {r[12]} |")
    out.append(f"\nTotal kernel time: {total * unit:.1f} us over {sum(r[1] for r in rows)} dispatches.")
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    text = summarise(a.db, a.top)
    if a.title:
        text = f"# {a.title}\n\n" + text
    sys.stdout.write(text + "\n")


if __name__ == "__main__":
    main()
