"""Summarise rocprofv3 ``--pmc`` passes (``--output-format csv``, one directory per pass) into a
per-kernel markdown table for ``profiles/``.

Each pass directory holds ``*_counter_collection.csv`` (one row per dispatch x counter). The
counters of all passes are averaged per kernel over its dispatches, then combined:

* LDS bank-conflict rate = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles / LDS cycles);
* wave time split: SQ_WAIT_ANY (parked on s_waitcnt / barrier), SQ_WAIT_INST_ANY (issue stall),
  SQ_ACTIVE_INST_ANY (issuing), as shares of their sum;
* HBM-side bytes: FETCH_SIZE is doubled (on gfx950 it reports half the bytes of wide
  coalesced reads, MI355X_MICROARCH.md) plus WRITE_SIZE, divided by the pass-1 duration;
* L2 hit rate = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum);
* MFMA: SQ_INSTS_MFMA per dispatch and SQ_VALU_MFMA_BUSY_CYCLES.

    python tools/pmc_summary.py gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3 --title ...
"""

import argparse
import collections
import csv
import glob
import os


def load(dirs):
    per = collections.defaultdict(lambda: collections.defaultdict(list))  # kernel -> counter -> values
    dur = collections.defaultdict(list)
    meta = {}
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            seen = set()
            with open(path) as fh:
                for row in csv.DictReader(fh):
                    k = row["Kernel_Name"].split("(")[0].replace("void ", "")
                    per[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
                    key = (path, row["Dispatch_Id"])
                    if key not in seen:
                        seen.add(key)
                        dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-3)
                        meta[k] = (row["Grid_Size"], row["Workgroup_Size"], row["LDS_Block_Size"], row["VGPR_Count"],
                                   row["SGPR_Count"])
    return per, dur, meta


def mean(xs):
    return sum(xs) / len(xs) if xs else float("nan")


def summarise(dirs, title, prefix="mislo::"):
    per, dur, meta = load(dirs)
    rows = []
    for k, c in per.items():
        if prefix and not k.startswith(prefix):
            continue
        g = lambda n: mean(c.get(n, []))  # noqa: E731
        t_us = min(dur[k]) if dur[k] else float("nan")  # least-perturbed dispatch under PMC
        lds = g("SQ_LDS_IDX_ACTIVE")
        w_any, w_inst, act = g("SQ_WAIT_ANY"), g("SQ_WAIT_INST_ANY"), g("SQ_ACTIVE_INST_ANY")
        tot = w_any + w_inst + act
        hbm = 2 * g("FETCH_SIZE") * 1024 + g("WRITE_SIZE") * 1024
        hit, miss = g("TCC_HIT_sum"), g("TCC_MISS_sum")
        waves = g("SQ_WAVES")
        rows.append((k, len(c.get("SQ_WAVES", [])), t_us, waves,
                     g("SQ_INSTS_VALU") / waves if waves else float("nan"),
                     g("SQ_INSTS_LDS") / waves if waves else float("nan"),
                     100 * g("SQ_LDS_BANK_CONFLICT") / lds if lds else 0.0,
                     100 * w_any / tot if tot else float("nan"), 100 * w_inst / tot if tot else float("nan"),
                     100 * act / tot if tot else float("nan"),
                     hbm / 1e6, hbm / (t_us * 1e3) if t_us else float("nan"),
                     100 * hit / (hit + miss) if hit + miss else float("nan"),
                     g("SQ_INSTS_MFMA"), g("SQ_VALU_MFMA_BUSY_CYCLES"), meta.get(k)))
    rows.sort(key=lambda r: -r[2] * r[1])
    out = [f"# {title}", "",
           "| kernel | dispatches | min us | waves | VALU/wave | LDS/wave | LDS conflict % | wait % | "
           "issue-stall % | active % | HBM MB | GB/s | L2 hit % | MFMA insts | MFMA busy cyc | grid/wg/lds/vgpr/sgpr |",
           "|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        m = "/".join(r[15]) if r[15] else ""
        out.append(f"| `{r[0]}` | {r[1]} | {r[2]:.1f} | {r[3]:.0f} | {r[4]:.1f} | {r[5]:.1f} | {r[6]:.2f} | "
                   f"{r[7]:.1f} | {r[8]:.1f} | {r[9]:.1f} | {r[10]:.2f} | {r[11]:.0f} | {r[12]:.1f} | {r[13]:.0f} | "
                   f"{r[14]:.0f} | {m} |")
    out.append("")
    out.append("Durations are from the PMC passes (the profiler serialises dispatches and adds overhead), so "
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
