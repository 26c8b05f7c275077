"""Where the agent's host memory goes: RSS / private anon after each step of bringing up the
native window engine (no torch), for the agent's default capacities."""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def anon_mb() -> float:
    tot, cur = 0, False
    with open("/proc/self/smaps") as f:
        for ln in f:
            p = ln.split()
            if p and "-" in p[0] and not p[0].endswith(":"):
                cur = len(p) <= 5
            elif p and p[0] == "Rss:" and cur:
                tot += int(p[1])
    return tot / 1024


def rss_mb() -> float:
    with open("/proc/self/statm") as f:
        return int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE") / 2**20


def big_anon(min_mb: float = 8.0):
    """Anonymous mappings with >= min_mb resident: (size MB, rss MB, flags)."""
    out, cur = [], None
    with open("/proc/self/smaps") as f:
        for ln in f:
            p = ln.split()
            if p and "-" in p[0] and not p[0].endswith(":"):
                a, b = (int(x, 16) for x in p[0].split("-"))
                cur = [(b - a) / 2**20, 0.0, p[1]] if len(p) <= 5 else None
                if cur is not None:
                    out.append(cur)
            elif p and p[0] == "Rss:" and cur is not None:
                cur[1] = int(p[1]) / 1024
    return sorted([m for m in out if m[1] >= min_mb], key=lambda m: -m[1])


def top_mappings(n: int = 6, min_mb: float = 4.0):
    """The largest resident mappings (RSS >= min_mb): (rss MB, kind, name)."""
    out, cur = [], None
    with open("/proc/self/smaps") as f:
        for ln in f:
            p = ln.split()
            if p and "-" in p[0] and not p[0].endswith(":"):
                name = " ".join(p[5:]) if len(p) > 5 else "[anon]"
                cur = [0.0, p[1], name]
                out.append(cur)
            elif p and p[0] == "Rss:" and cur is not None:
                cur[0] = int(p[1]) / 1024
    agg = {}
    for rss, flags, name in out:
        key = (os.path.basename(name) if name.startswith("/") else name)
        agg[key] = agg.get(key, 0.0) + rss
    return sorted([(v, k) for k, v in agg.items() if v >= min_mb], reverse=True)[:n]


def step(name, detail=False):
    print(f"{name:40s} rss {rss_mb():8.1f} MB  anon {anon_mb():8.1f} MB", flush=True)
    if detail:
        for rss, key in top_mappings():
            print(f"      {rss:8.1f} MB  {key}", flush=True)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_250_000
    print("env:", {k: v for k, v in os.environ.items() if k.startswith(("GPU_", "HSA_", "HIP_", "ROC_"))}, flush=True)
    step("start")
    from llm_slo_ebpf_toolkit_amd.ops import load_agent

    mod = load_agent(init=False)
    step("import _mislo_agent")
    mod.device_count()
    step("hip runtime init (device_count)")
    load_agent()
    step("set_tables", detail=True)
    from llm_slo_ebpf_toolkit_amd.pipeline.window import WindowPipeline

    small = WindowPipeline(65536, 4096, 64, 0, None, model="bayes", learn=False, user_cap=16384)
    step("WindowPipeline(sig_cap=65536)")
    small.eng.close()
    del small
    step("  closed")
    pipe = WindowPipeline(n, 16384, 64, 0, None, model="bayes", learn=False, user_cap=n // 4)
    step(f"WindowPipeline(sig_cap={n})")
    for m in big_anon():
        print(f"    anon mapping {m[0]:9.1f} MB  rss {m[1]:8.1f} MB  {m[2]}", flush=True)
    from llm_slo_ebpf_toolkit_amd.collector import bpf

    names = bpf.RingNames.of(f"/mislo-rss-{os.getpid()}")
    # the agent's replay-source sizes: two windows of framed records, a window of USER24 records
    ring, user, spans = bpf.create_rings(names, 2 * 24 * 1_000_000, 1_000_000, 4 * 16384)
    step("create_rings")
    from llm_slo_ebpf_toolkit_amd.pipeline.window import RingWindowSource

    src = RingWindowSource(pipe, ring, user, spans)
    step("register rings (hipHostRegister)")
    for _ in range(4):
        src.step(64)
    src.drain()
    step("4 empty windows", detail=True)
    # real windows (spans only: the join, posterior, refit and result paths run), the queue save
    # areas counted after each phase: which call maps a hardware queue beyond the first stream's
    import numpy as np

    from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator

    def areas():
        return len([m for m in big_anon(100.0) if 170 < m[0] < 180])

    w = ReplayGenerator(ReplayConfig(events_per_window=4096, spans_per_window=4096, n_services=64)).next_window()
    sp = np.ascontiguousarray(w.spans)
    for k in range(6):
        j = pipe.submit([], [], [(sp.ctypes.data, sp.nbytes)], 64, labels=np.zeros(64, np.int32))
        print(f"  window {j} submitted: queue areas {areas()}", flush=True)
        pipe.wait(j)
        print(f"  window {j} done:      queue areas {areas()}", flush=True)
        pipe.results(j, 64)
        print(f"  window {j} results:   queue areas {areas()}", flush=True)
    step("6 span windows", detail=True)
    pipe.eng.close()
    step("engine closed")


if __name__ == "__main__":
    main()
