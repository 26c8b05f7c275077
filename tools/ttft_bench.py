"""TTFT / tokens-per-second of the random-init Llama workload on MI355X (configs 2-4).

  python tools/ttft_bench.py --preset 7b --batch 1 --prompt 512 --new 64 --iters 5
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/ttft_bench.py --preset 7b

Run it with ROCP_TOOL_LIBRARIES=llm_slo_ebpf_toolkit_amd/probes/rocprof/libmislo_rocprof.so
to feed the agent's ring with the workload's GPU signals. Prints one JSON line.
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="7b")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--new", type=int, default=64)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    a = ap.parse_args()
    from llm_slo_ebpf_toolkit_amd.parallel import dist as pdist

    env = pdist.env()
    pg = pdist.init()
    torch.cuda.set_device(env.local_rank)
    dev = torch.device("cuda", env.local_rank)
    if env.world > 1:
        from llm_slo_ebpf_toolkit_amd.parallel.tensor import build_tp

        model = build_tp(a.preset, env.rank, env.world, dev, group=pg)
    else:
        from llm_slo_ebpf_toolkit_amd.models.llama import build

        model = build(a.preset, dev)
    g = torch.Generator(device="cpu").manual_seed(1)
    prompt = torch.randint(0, model.cfg.vocab, (a.batch, a.prompt), generator=g).to(dev)
    for _ in range(a.warmup):
        model.generate(prompt, 4)
    runs = [model.generate(prompt, a.new) for _ in range(a.iters)]
    ttft = [r["ttft_ms"] for r in runs]
    tps = [r["tokens_per_s"] for r in runs]
    if env.rank == 0:
        print(json.dumps({"preset": a.preset, "params_b": round(model.cfg.params() / 1e9, 2), "tp": env.world,
                          "batch": a.batch, "prompt_tokens": a.prompt, "new_tokens": a.new,
                          "ttft_ms_p50": round(float(np.median(ttft)), 3), "ttft_ms_max": round(max(ttft), 3),
                          "decode_tokens_per_s_p50": round(float(np.median(tps)), 1),
                          "hbm_gib": round(torch.cuda.max_memory_allocated(dev) / 2**30, 2)}), flush=True)
    pdist.destroy()


if __name__ == "__main__":
    main()
