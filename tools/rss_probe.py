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


def step(name):
    print(f"{name:40s} rss {rss_mb():8.1f} MB  anon {anon_mb():8.1f} MB", flush=True)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_250_000
    step("start")
    from llm_slo_ebpf_toolkit_amd.ops import load_agent

    mod = load_agent(init=False)
    step("import _mislo_agent")
    mod.device_count()
    step("hip runtime init (device_count)")
    load_agent()
    step("set_tables")
    from llm_slo_ebpf_toolkit_amd.pipeline.window import WindowPipeline

    pipe = WindowPipeline(n, 16384, 64, 0, None, model="bayes", learn=False, user_cap=n // 4)
    step(f"WindowPipeline(sig_cap={n})")
    from llm_slo_ebpf_toolkit_amd.collector import bpf

    names = bpf.RingNames.of(f"/mislo-rss-{os.getpid()}")
    ring, user, spans = bpf.create_rings(names, 4 * 24 * 1_000_000, 4_000_000, 4 * 16384)
    step("create_rings")
    from llm_slo_ebpf_toolkit_amd.pipeline.window import RingWindowSource

    src = RingWindowSource(pipe, ring, user, spans)
    step("register rings (hipHostRegister)")
    for _ in range(4):
        src.step(64)
    src.drain()
    step("4 empty windows")
    pipe.eng.close()
    step("engine closed")


if __name__ == "__main__":
    main()
