"""Summarise rocprofv3 ``--pmc`` passes (``--output-format csv``, one directory per pass) into a
per-kernel, per-launch-shape markdown table for ``profiles/``.

Each pass directory holds ``*_counter_collection.csv`` (one row per dispatch x counter). Rows
are grouped by kernel AND launch shape (grid / workgroup / LDS): a kernel launched in several
phases (e.g. ``k_probe`` over the window's rows, then over the imported rows) gets one row per
phase. Every rate is computed PER DISPATCH from that dispatch's own counters and duration (the
counters of one pass and the timestamps of the same dispatch) and the table reports the median
over dispatches -- never pooled bytes over a pooled minimum duration:

* LDS bank-conflict rate = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles / LDS cycles);
* wave time split: SQ_WAIT_ANY (parked on s_waitcnt / barrier), SQ_WAIT_INST_ANY (issue stall),
  SQ_ACTIVE_INST_ANY (issuing), as shares of their sum;
* HBM-side read GB/s = 2 x FETCH_SIZE (gfx950 reports half the bytes of wide coalesced reads,
  MI355X_MICROARCH.md) / duration of the same dispatch; write GB/s = WRITE_SIZE / duration;
* L2 hit rate = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum);
* MFMA: SQ_INSTS_MFMA per dispatch and SQ_VALU_MFMA_BUSY_CYCLES.

Durations under PMC are inflated (the profiler serialises dispatches), so every GB/s here is a
lower bound of the unprofiled kernel's; the unprofiled per-dispatch times come from the
``--kernel-trace`` run (``tools/kernel_phases.py``).

    python tools/pmc_summary.py gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3 --title ...
"""

import argparse
import collections
import csv
import glob
import os
import statistics


def load(dirs):
    """-> {(kernel, shape): [dispatch dicts {counter: value, "_us": duration}]} per pass dir."""
    groups = collections.defaultdict(list)
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            disp = {}
            with open(path) as fh:
                for row in csv.DictReader(fh):
                    k = row["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
                    shape = (row["Grid_Size"], row["Workgroup_Size"], row["LDS_Block_Size"], row["VGPR_Count"],
                             row["SGPR_Count"])
                    key = (path, row["Dispatch_Id"])
                    e = disp.get(key)
                    if e is None:
                        e = disp[key] = {"_k": (k, shape),
                                         "_us": (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-3}
                    e[row["Counter_Name"]] = e.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
            for e in disp.values():
                groups[e.pop("_k")].append(e)
    return groups


def med(xs):
    xs = [x for x in xs if x == x]
    return statistics.median(xs) if xs else float("nan")


def per_dispatch(ds, fn):
    out = []
    for d in ds:
        try:
            out.append(fn(d))
        except (KeyError, ZeroDivisionError):
            continue
    return out


def summarise(dirs, title, prefix="mislo::"):
    groups = load(dirs)
    by_kernel = collections.defaultdict(dict)
    for (k, shape), ds in groups.items():
        if prefix and not k.startswith(prefix):
            continue
        by_kernel[(k, shape)] = ds
    rows = []
    for (k, shape), ds in by_kernel.items():
        us = [d["_us"] for d in ds]
        lds = per_dispatch(ds, lambda d: 100 * d["SQ_LDS_BANK_CONFLICT"] / d["SQ_LDS_IDX_ACTIVE"]
                           if d["SQ_LDS_IDX_ACTIVE"] else 0.0)
        split = per_dispatch(ds, lambda d: (d["SQ_WAIT_ANY"], d["SQ_WAIT_INST_ANY"], d["SQ_ACTIVE_INST_ANY"]))
        tot = [sum(s) for s in split]
        rd = per_dispatch(ds, lambda d: 2 * d["FETCH_SIZE"] * 1024 / (d["_us"] * 1e3))
        wr = per_dispatch(ds, lambda d: d["WRITE_SIZE"] * 1024 / (d["_us"] * 1e3))
        mb = per_dispatch(ds, lambda d: (2 * d["FETCH_SIZE"]) * 1024 / 1e6)
        hit = per_dispatch(ds, lambda d: 100 * d["TCC_HIT_sum"] / (d["TCC_HIT_sum"] + d["TCC_MISS_sum"]))
        waves = per_dispatch(ds, lambda d: d["SQ_WAVES"])
        valu = per_dispatch(ds, lambda d: d["SQ_INSTS_VALU"] / d["SQ_WAVES"])
        ldsi = per_dispatch(ds, lambda d: d["SQ_INSTS_LDS"] / d["SQ_WAVES"])
        mfma = per_dispatch(ds, lambda d: d["SQ_INSTS_MFMA"])
        rows.append((k, shape, len(ds), med(us), min(us), max(us), med(waves), med(valu), med(ldsi), med(lds),
                     med([100 * s[0] / t for s, t in zip(split, tot) if t]),
                     med([100 * s[1] / t for s, t in zip(split, tot) if t]),
                     med([100 * s[2] / t for s, t in zip(split, tot) if t]),
                     med(mb), med(rd), med(wr), med(hit), med(mfma)))
    rows.sort(key=lambda r: -r[3] * r[2])
    out = [f"# {title}", "",
           "One row per kernel and launch shape (grid/wg/lds/vgpr/sgpr); every rate is per dispatch (its own "
           "counters over its own duration), median over dispatches.", "",
           "| kernel | grid/wg/lds/vgpr/sgpr | dispatches | median us | min-max us | waves | VALU/wave | LDS/wave | "
           "LDS conflict % | wait % | issue-stall % | active % | read MB | read GB/s | write GB/s | L2 hit % | MFMA |",
           "|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|"]
    f = lambda v, p=1: "" if v != v else f"{v:.{p}f}"  # noqa: E731
    for r in rows:
        out.append(f"| `{r[0]}` | {'/'.join(r[1])} | {r[2]} | {f(r[3])} | {f(r[4])}-{f(r[5])} | {f(r[6], 0)} | "
                   f"{f(r[7])} | {f(r[8])} | {f(r[9], 2)} | {f(r[10])} | {f(r[11])} | {f(r[12])} | {f(r[13], 2)} | "
                   f"{f(r[14], 0)} | {f(r[15], 0)} | {f(r[16])} | {f(r[17], 0)} |")
    out.append("")
    out.append("Durations are from the PMC passes (the profiler serialises dispatches and adds overhead), so every "
               "GB/s is a lower bound. FETCH_SIZE is doubled for gfx950's half-count of wide coalesced reads.")
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--title", default="rocprofv3 PMC summary")
    ap.add_argument("--prefix", default="mislo::")
    a = ap.parse_args()
    print(summarise(a.dirs, a.title, a.prefix))


if __name__ == "__main__":
    main()
