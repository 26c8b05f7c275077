"""Does device memory (hipMalloc) show up in this process's RSS? Allocates device buffers
through libamdhip64 (ctypes) in the engine's sizes (the 256 MiB context table, the 128 MiB
trace-id table, ~51 MiB window buffers) and in 1 GiB blocks, with and without hipMemset,
printing RSS (anon / file / shmem) after each step."""

import ctypes
import os


def status() -> dict:
    out = {}
    with open("/proc/self/status") as f:
        for ln in f:
            if ln.startswith(("VmRSS", "RssAnon", "RssFile", "RssShmem")):
                k, v = ln.split(":")
                out[k] = int(v.split()[0]) / 1024
    return out


def show(tag):
    s = status()
    print(f"{tag:40s} rss {s['VmRSS']:8.1f}  anon {s['RssAnon']:8.1f}  file {s['RssFile']:7.1f}  "
          f"shmem {s['RssShmem']:7.1f} MB", flush=True)


hip = ctypes.CDLL("libamdhip64.so")
show("start")
n = ctypes.c_int()
hip.hipGetDeviceCount(ctypes.byref(n))
hip.hipSetDevice(0)
hip.hipDeviceSynchronize()
show("runtime up")


def alloc(size, memset, tag):
    p = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(size)) == 0
    show(f"{tag}: hipMalloc")
    if memset:
        assert hip.hipMemset(p, 0, ctypes.c_size_t(size)) == 0
        hip.hipDeviceSynchronize()
        show(f"{tag}: hipMemset")
    return p


bufs = [alloc(64 << 20, False, "64 MiB no memset"),
        alloc(256 << 20, False, "256 MiB no memset"),
        alloc(256 << 20, True, "256 MiB + memset"),
        alloc(128 << 20, True, "128 MiB + memset"),
        alloc(51 << 20, True, "51 MiB + memset"),
        alloc(51 << 20, True, "51 MiB + memset (2)"),
        alloc(1 << 30, True, "1 GiB + memset"),
        alloc(1 << 30, True, "1 GiB + memset (2)")]
for p in bufs:
    hip.hipFree(p)
hip.hipDeviceSynchronize()
show("freed")
