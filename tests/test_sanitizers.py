"""Host ring code under sanitizers (SURVEY §5 race detection): the
multi-producer stress harness (tests/native/ring_stress.cpp) built with AddressSanitizer +
UBSan and with ThreadSanitizer -- HostRing producers racing a wrapping consumer, kernel-layout
BPF ring reserve / commit / discard / output from several threads against the consumer,
multi-threaded framed appends and parallel consumption."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RT = os.path.join(ROOT, "llm_slo_ebpf_toolkit_amd", "runtime", "csrc")
SRCS = [os.path.join(ROOT, "tests", "native", "ring_stress.cpp")] + \
       [os.path.join(RT, f) for f in ("ring.cpp", "bpfring.cpp", "pool.cpp")]


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.timeout(600)
@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_ring_stress_under_sanitizer(san, tmp_path):
    exe = tmp_path / "ring_stress"
    flags = ["-std=c++17", "-O1", "-g", "-pthread", f"-fsanitize={san}", "-fno-omit-frame-pointer", f"-I{RT}"]
    subprocess.run(["g++", *flags, *SRCS, "-o", str(exe), "-lrt"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", TSAN_OPTIONS="halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=500)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "ring stress ok" in r.stdout
    assert "Sanitizer" not in r.stderr, r.stderr[-4000:]
