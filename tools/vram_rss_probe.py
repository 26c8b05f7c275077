"""Does device memory (hipMalloc) show up in this process's RSS, and does it consume host
RAM? Allocates and touches device buffers through libamdhip64 (ctypes) and prints RSS and
the system's MemAvailable before and after."""

import ctypes
import os


def meminfo(key: str) -> float:
    with open("/proc/meminfo") as f:
        for ln in f:
            if ln.startswith(key + ":"):
                return int(ln.split()[1]) / 1024
    return -1.0


def rss() -> float:
    with open("/proc/self/statm") as f:
        return int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE") / 2**20


def show(tag):
    print(f"{tag:28s} rss {rss():9.1f} MB   MemAvailable {meminfo('MemAvailable'):10.1f} MB", flush=True)


hip = ctypes.CDLL("libamdhip64.so")
show("start")
n = ctypes.c_int()
hip.hipGetDeviceCount(ctypes.byref(n))
hip.hipSetDevice(0)
hip.hipDeviceSynchronize()
show("runtime up")
bufs = []
for i in range(4):
    p = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 30)) == 0
    assert hip.hipMemset(p, 1, ctypes.c_size_t(1 << 30)) == 0
    bufs.append(p)
    hip.hipDeviceSynchronize()
    show(f"{i + 1} GiB device allocated")
for p in bufs:
    hip.hipFree(p)
hip.hipDeviceSynchronize()
show("freed")
