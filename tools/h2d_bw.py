"""Pinned host -> device bandwidth on one MI355X: one copy per window vs the same bytes split
into k concurrent copies on k streams (several SDMA engines), for the window sizes the
pipeline moves (diagnostic; results in profiles/h2d_bw_r1.log)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def run(nbytes: int, k: int, reps: int = 20) -> float:
    dev = torch.device("cuda", 0)
    host = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    streams = [torch.cuda.Stream(dev) for _ in range(k)]
    q = nbytes // k
    for it in range(reps + 3):
        if it == 3:
            torch.cuda.synchronize()
            t = time.perf_counter()
        for j, s in enumerate(streams):
            hi = nbytes if j == k - 1 else (j + 1) * q
            with torch.cuda.stream(s):
                d[j * q:hi].copy_(host[j * q:hi], non_blocking=True)
        for s in streams:
            s.synchronize()
    return reps * nbytes / (time.perf_counter() - t) / 1e9


def main():
    for mb in (16, 24, 32, 64):
        print(f"{mb} MiB:", "  ".join(f"{k} stream(s) {run(mb << 20, k):.1f} GB/s" for k in (1, 2, 4)), flush=True)


if __name__ == "__main__":
    main()
