"""Host-side issue latency of pinned H2D copies (diagnostic).

Times how long the host blocks in each call of a WindowPipeline-like copy sequence, with
the copy engine idle and with a previous copy still in flight."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    n = 32 << 20
    dev = torch.device("cuda", 0)
    host = [torch.empty(n, dtype=torch.uint8).pin_memory() for _ in range(2)]
    small = torch.empty(int(os.environ.get("SMALL", 1 << 20)), dtype=torch.uint8).pin_memory()
    d = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(2)]
    ds = torch.empty(small.numel(), dtype=torch.uint8, device=dev)
    cs = torch.cuda.Stream(dev)
    ks = torch.cuda.Stream(dev)
    ev = [torch.cuda.Event() for _ in range(2)]
    torch.cuda.synchronize()
    for mode in ("torch_copy", "torch_copy_chunked4", "slice_copy"):
        res = []
        for i in range(12):
            b = i % 2
            t0 = time.perf_counter()
            cs.wait_event(ev[b])
            t1 = time.perf_counter()
            with torch.cuda.stream(cs):
                if mode == "torch_copy":
                    d[b].copy_(host[b], non_blocking=True)
                elif mode == "torch_copy_chunked4":
                    q = n // 4
                    for j in range(4):
                        d[b][j * q:(j + 1) * q].copy_(host[b][j * q:(j + 1) * q], non_blocking=True)
                else:
                    d[b][: n - 7].copy_(host[b][: n - 7], non_blocking=True)
                t2 = time.perf_counter()
                ds.copy_(small, non_blocking=True)
                t3 = time.perf_counter()
                ev[b].record(cs)
            t4 = time.perf_counter()
            res.append((1e6 * (t1 - t0), 1e6 * (t2 - t1), 1e6 * (t3 - t2), 1e6 * (t4 - t3)))
        torch.cuda.synchronize()
        print(mode, "wait/big/small/record us per call:")
        for r in res:
            print("   " + " ".join(f"{x:8.1f}" for x in r))
    # bandwidth
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(10):
        with torch.cuda.stream(cs):
            d[i % 2].copy_(host[i % 2], non_blocking=True)
    torch.cuda.synchronize()
    print(f"H2D {10 * n / (time.perf_counter() - t) / 1e9:.1f} GB/s (one stream)")
    cs2 = torch.cuda.Stream(dev)
    t = time.perf_counter()
    for i in range(10):
        with torch.cuda.stream(cs if i % 2 else cs2):
            d[i % 2].copy_(host[i % 2], non_blocking=True)
    torch.cuda.synchronize()
    print(f"H2D {10 * n / (time.perf_counter() - t) / 1e9:.1f} GB/s (two streams)")


if __name__ == "__main__":
    main()
