"""In-tree build of the native extensions with hipcc for gfx950 (no hipify, no JIT cache).

Produces, next to the sources (so the .so travels with the repo snapshot to the GPU box):

* ``ops/_mislo_hip<EXT_SUFFIX>``    -- torch extension: decode / join / posterior kernels
  and the ``Engine`` bindings (hipcc, --offload-arch=gfx950).
* ``ops/_mislo_agent<EXT_SUFFIX>``  -- the native window engine (HIP + RCCL, pybind11, no
  torch): what the agent daemon and the benchmark run.
* ``probes/rocprof/libmislo_rocprof.so`` -- rocprofiler-sdk tool library (GPU signals
  from inside LLM workloads into the agent's shared-memory ring).
* ``runtime/_mislo_rt<EXT_SUFFIX>`` -- native runtime (pinned MPSC ring, replay generator,
  gate statistics on the host) exposed through pybind11; also ``runtime/libmislo_rt.so``
  with a C ABI for external producers (BPF loader, rocprofiler-sdk tool).

Usage: ``python -m llm_slo_ebpf_toolkit_amd.ops.build [--force] [-j N]``.
Object files are rebuilt only when a source or header is newer.
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from typing import List, Sequence

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
RT_CSRC = os.path.join(PKG, "runtime", "csrc")
BUILD = os.path.join(PKG, "_build")
ARCH = os.environ.get("MISLO_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"

HIP_SOURCES = ["decode.hip", "join.hip", "posterior.hip", "gatestats.hip", "storm.hip", "exchange.hip"]
RT_SOURCES = ["ring.cpp", "replay.cpp", "pool.cpp", "bpfring.cpp", "probesim.cpp", "tables.cpp", "assemble.cpp",
              "bpfsys.cpp", "procsampler.cpp", "gpusampler.cpp", "rt_bindings.cpp"]


def torch_flags():
    import torch
    import torch.utils.cpp_extension as ce

    inc = ce.include_paths()
    libdir = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cflags = [f"-I{p}" for p in inc] + [
        f"-I{sysconfig.get_paths()['include']}", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DTORCH_API_INCLUDE_EXTENSION_H", "-DTORCH_EXTENSION_NAME=_mislo_hip", "-DUSE_ROCM",
        "-D__HIP_PLATFORM_AMD__=1",
    ]
    ldflags = [f"-L{libdir}", f"-Wl,-rpath,{libdir}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
               "-ltorch_hip", "-ltorch_python"]
    return cflags, ldflags


def pybind_flags():
    import pybind11

    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def _newer(target: str, deps: Sequence[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _headers(d: str) -> List[str]:
    return [os.path.join(d, f) for f in os.listdir(d) if f.endswith(".h")]


def _run(cmd: List[str]) -> None:
    print("+", " ".join(cmd[:6]), "...", flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout)
        raise RuntimeError(f"build step failed: {' '.join(cmd)}")


def build_hip_ext(force: bool = False, jobs: int = 4) -> str:
    os.makedirs(BUILD, exist_ok=True)
    out = os.path.join(HERE, "_mislo_hip" + EXT_SUFFIX)
    hdrs = _headers(CSRC)
    tflags, tld = torch_flags()
    common = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result"]
    # extra -D flags for diagnostic builds (e.g. MISLO_HIP_DEFINES=-DMISLO_PROBE_PROFILE, with force)
    common += os.environ.get("MISLO_HIP_DEFINES", "").split()
    jobs_list = []
    objs = []
    for src in HIP_SOURCES:
        path = os.path.join(CSRC, src)
        if not os.path.exists(path):
            continue
        obj = os.path.join(BUILD, src + ".o")
        objs.append(obj)
        if force or _newer(obj, [path] + hdrs):
            jobs_list.append([HIPCC, *common, "-c", path, "-o", obj])
    bind = os.path.join(CSRC, "bindings.cpp")
    bobj = os.path.join(BUILD, "bindings.o")
    objs.append(bobj)
    if force or _newer(bobj, [bind] + hdrs):
        jobs_list.append([HIPCC, *common, "-x", "hip", *tflags, "-c", bind, "-o", bobj])
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(_run, jobs_list))
    if force or jobs_list or _newer(out, objs):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", out, *tld,
              f"-L{ROCM}/lib", "-lamdhip64"])
    return out


AGENT_KERNELS = ["decode.hip", "join.hip", "posterior.hip", "exchange.hip"]


def build_agent_ext(force: bool = False, jobs: int = 4) -> str:
    """``_mislo_agent``: the native window engine (engine.hip) + the window kernels, bound with
    pybind11 and linked against the HIP runtime and RCCL only (no PyTorch)."""
    os.makedirs(BUILD, exist_ok=True)
    out = os.path.join(HERE, "_mislo_agent" + EXT_SUFFIX)
    hdrs = _headers(CSRC)
    common = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result"]
    common += os.environ.get("MISLO_HIP_DEFINES", "").split()
    jobs_list, objs = [], []
    for src in AGENT_KERNELS:  # shared with the torch extension (same flags, same objects)
        objs.append(os.path.join(BUILD, src + ".o"))
    eng = os.path.join(CSRC, "engine.hip")
    eobj = os.path.join(BUILD, "engine.hip.o")
    objs.append(eobj)
    if force or _newer(eobj, [eng] + hdrs):
        jobs_list.append([HIPCC, *common, "-c", eng, "-o", eobj])
    bind = os.path.join(CSRC, "agent_bindings.cpp")
    bobj = os.path.join(BUILD, "agent_bindings.o")
    objs.append(bobj)
    if force or _newer(bobj, [bind] + hdrs):
        jobs_list.append([HIPCC, *common, "-x", "hip", *pybind_flags(), "-c", bind, "-o", bobj])
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(_run, jobs_list))
    if force or jobs_list or _newer(out, objs):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", out, f"-L{ROCM}/lib", "-lamdhip64",
              "-lrccl", f"-Wl,-rpath,{ROCM}/lib"])
    return out


def build_runtime(force: bool = False, jobs: int = 4) -> List[str]:
    os.makedirs(BUILD, exist_ok=True)
    rt_dir = os.path.join(PKG, "runtime")
    hdrs = _headers(RT_CSRC)
    cxx = shutil.which("g++") or "c++"
    # -ffp-contract=off: the wire encoder's fixed-point values must match numpy bit for bit
    base = ["-O3", "-std=c++17", "-fPIC", "-pthread", "-Wall", "-ffp-contract=off", f"-I{ROCM}/include",
            "-D__HIP_PLATFORM_AMD__=1"]
    outs = []
    core = [os.path.join(RT_CSRC, s) for s in ("ring.cpp", "replay.cpp", "pool.cpp")]
    lib = os.path.join(rt_dir, "libmislo_rt.so")
    if force or _newer(lib, core + hdrs):
        _run([cxx, *base, "-shared", *core, "-o", lib])
    outs.append(lib)
    mod = os.path.join(rt_dir, "_mislo_rt" + EXT_SUFFIX)
    srcs = [os.path.join(RT_CSRC, s) for s in RT_SOURCES]
    if force or _newer(mod, srcs + hdrs):  # CPU only: no HIP runtime dependency
        _run([cxx, *base, *pybind_flags(), "-shared", *srcs, "-o", mod])
    outs.append(mod)
    return outs


def build_rocprof_tool(force: bool = False) -> str:
    """rocprofiler-sdk tool library (probes/rocprof): GPU signals -> shared-memory ring."""
    src = os.path.join(PKG, "probes", "rocprof", "mislo_rocprof.cpp")
    out = os.path.join(PKG, "probes", "rocprof", "libmislo_rocprof.so")
    rt_dir = os.path.join(PKG, "runtime")
    if force or _newer(out, [src, os.path.join(rt_dir, "libmislo_rt.so"),
                             os.path.join(PKG, "probes", "ebpf", "mislo_record.h")]):
        cxx = shutil.which("g++") or "c++"
        _run([cxx, "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", "-Wall", f"-I{ROCM}/include",
              f"-I{os.path.join(PKG, 'probes', 'ebpf')}", "-D__HIP_PLATFORM_AMD__=1", src, "-o", out,
              f"-L{rt_dir}", "-lmislo_rt", "-Wl,-rpath,$ORIGIN/../../runtime", f"-L{ROCM}/lib", "-lrocprofiler-sdk",
              f"-Wl,-rpath,{ROCM}/lib"])
    return out


def build_all(force: bool = False, jobs: int = 4) -> List[str]:
    outs = build_runtime(force, jobs)
    outs.append(build_hip_ext(force, jobs))
    outs.append(build_agent_ext(force, jobs))
    outs.append(build_rocprof_tool(force))
    return outs


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--only", choices=("hip", "agent", "runtime", "all"), default="all")
    a = ap.parse_args(argv)
    if a.only == "hip":
        outs = [build_hip_ext(a.force, a.jobs)]
    elif a.only == "agent":
        outs = [build_hip_ext(a.force, a.jobs), build_agent_ext(a.force, a.jobs)]
    elif a.only == "runtime":
        outs = build_runtime(a.force, a.jobs)
    else:
        outs = build_all(a.force, a.jobs)
    for o in outs:
        print("built", o)
    return 0


if __name__ == "__main__":
    sys.exit(main())
