"""xGMI link load for the config-4 interconnect fault: every GPU streams 256 MiB peer-to-peer
copies to every other GPU on its own streams, so every link of the node's full mesh carries
back-to-back DMA traffic and RCCL collectives queue behind it.

    python tools/xgmi_hog.py --gpus 8 --seconds 15
"""

import argparse
import time

import torch


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=torch.cuda.device_count())
    ap.add_argument("--seconds", type=float, default=15.0)
    ap.add_argument("--mib", type=int, default=256)
    a = ap.parse_args()
    n = min(a.gpus, torch.cuda.device_count())
    if n < 2:
        print("xgmi hog: fewer than 2 GPUs, nothing to load", flush=True)
        return 0
    elems = a.mib * (1 << 20) // 2
    src = [torch.ones(elems, dtype=torch.bfloat16, device=f"cuda:{i}") for i in range(n)]
    dst = {(i, j): torch.empty(elems, dtype=torch.bfloat16, device=f"cuda:{j}") for i in range(n) for j in range(n) if i != j}
    streams = {(i, j): torch.cuda.Stream(device=f"cuda:{i}") for (i, j) in dst}
    end = time.time() + a.seconds
    moved = 0
    print(f"xgmi hog on: {n} GPUs, {len(dst)} directed links", flush=True)
    while time.time() < end:
        for (i, j), d in dst.items():
            with torch.cuda.stream(streams[(i, j)]):
                d.copy_(src[i], non_blocking=True)
            moved += 2 * elems
        for i in range(n):
            torch.cuda.synchronize(i)
    print(f"xgmi hog off: {moved / 2**30:.1f} GiB moved", flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
