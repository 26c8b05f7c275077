"""The overhead guard's shedding ladder (safety.ShedLadder) acts on the window engine's real
sources: floors in mislo_cfg first (the producers stop emitting sub-threshold records), then the
procfs sampler's signals, then the GPU producers' drop mask, and only then probes (REF
cmd/agent/main.go:587-600 sheds by detaching a probe per over-budget tick)."""

import os

import numpy as np

from llm_slo_ebpf_toolkit_amd.collector import bpf
from llm_slo_ebpf_toolkit_amd.collector import procfs
from llm_slo_ebpf_toolkit_amd.runtime import load
from llm_slo_ebpf_toolkit_amd.safety import ShedLadder
from llm_slo_ebpf_toolkit_amd.signals import catalog


class FakeSampler:
    def __init__(self):
        self.mask, self.paused = procfs.ALL_MASK, False


class FakeProbes:
    def __init__(self):
        self.left = ["tls_handshake_ms", "syscall_latency_ms"]

    def shed_next(self):
        return self.left.pop(0) if self.left else None


def test_ladder_order_floors_sampler_gpu_probes():
    rt = load()
    name = f"/mislo-shed-{os.getpid()}"
    names = bpf.RingNames.of(name)
    ring, user, spans = bpf.create_rings(names, 1 << 16, 1024, 1024)
    maps = bpf.EmulatedMaps(ring)
    s, pm = FakeSampler(), FakeProbes()
    lad = ShedLadder(catalog.DISABLE_ORDER, maps=maps, sampler=s, user_ring=user, probe_manager=pm)
    steps = []
    while True:
        w = lad.step()
        if w is None:
            break
        steps.append(w)
    kinds = [w.split(":")[0] for w in steps]
    assert kinds[0] == "floors"
    assert kinds[1:5] == ["sampler"] * 4 and s.paused and s.mask == 0
    assert kinds[5:9] == ["gpu"] * 4 and kinds[9:] == ["probe", "probe"]
    # floors: every kernel probe signal now emits only at or above its evidence threshold
    for spec in catalog.SIGNALS:
        if not spec.gpu and 0 < spec.kernel_type < 120:
            assert maps.cfg_get(bpf.cfg_floor(spec.kernel_type)) == round(spec.elevated / spec.decode_scale)
    # the sampler sheds in REF's cost order: runqueue before steal before mem reclaim before cfs
    assert [w.split(":")[1] for w in steps[1:5]] == ["runqueue_delay_ms", "mem_reclaim_latency_ms", "cpu_steal_pct",
                                                     "cfs_throttled_ms"]
    gpu_types = {catalog.BY_NAME[n].kernel_type for n in catalog.GPU_SIGNALS}
    assert user.drop_mask == sum(1 << t for t in gpu_types)
    assert lad.disabled() >= set(procfs.SIGNAL_TYPES) | set(catalog.GPU_SIGNALS) | {"tls_handshake_ms"}
    del ring, user, spans, rt


class OverBudget:
    """An overhead guard that always reads over budget (the CPU test cannot load a box)."""

    source = None

    def evaluate(self):
        return 50.0, True


def test_forced_over_budget_raises_floors_and_the_next_windows_carry_fewer_events():
    """The agent's window loop with the replay producer (ProbeSim applies mislo_cfg floors per
    record, as the BPF probes do): the first over-budget tick raises the floors, and the windows
    after it carry far fewer kernel records than the one before."""
    from llm_slo_ebpf_toolkit_amd.agent.daemon import Agent, AgentOptions

    o = AgentOptions(engine="cpu", source="replay", gpus=1, window_events=8192, window_spans=256, window_groups=8,
                     window_ms=300, metrics_bind="", output="stdout", ring_name=f"/mislo-shedw-{os.getpid()}",
                     config="", min_confidence=0.0, scenario="baseline")
    import io

    a = Agent(o, out_stream=io.StringIO())
    a.guard = OverBudget()
    seen = []
    orig = a.metrics.observe_window

    def spy(hist, status, dbg, n_events, *args, **kw):
        seen.append(int(n_events))
        return orig(hist, status, dbg, n_events, *args, **kw)

    a.metrics.observe_window = spy
    rc = a.run_windows(max_windows=8)
    a.close()
    assert rc == 0 and len(seen) >= 6, seen
    assert a.ladder.shed and a.ladder.shed[0].startswith("floors:")
    # (the first window may be partial: the producer's staged batches of the window it was cut
    # in flush at the producer's own window end, into the agent's next window)
    before, after = max(seen[:2]), np.mean(seen[-3:])
    assert after < 0.6 * before, seen
