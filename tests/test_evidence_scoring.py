"""The config 2/3/4 evidence harnesses' per-window scoring (tools/config3_evidence.py score)."""

import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

from config3_evidence import phase_windows, score  # noqa: E402

S = 1_000_000_000


def _attr(t, dom, svc="rag-service"):
    return (t + S // 10, {"incident_id": f"gpu-{t}-000", "service": svc, "predicted_fault_domain": dom,
                          "fault_hypotheses": []})


def test_phase_windows_follow_the_agents_grid():
    # a 15 s phase starting 0.14 s after a cut holds 14 whole windows: (0.86, 1.86] ... (13.86, 14.86]
    wins = phase_windows(0, 15 * S, S, cuts=[-S * 14 // 100])
    assert len(wins) == 14 and wins[0] == 186 * S // 100 and wins[-1] == 1486 * S // 100
    # phase starting on a cut: 15; no grid known: counted from the phase start
    assert len(phase_windows(0, 15 * S, S, cuts=[7 * S])) == 15
    assert len(phase_windows(0, 15 * S, S)) == 15


def test_score_counts_misses_against_whole_windows_only():
    cuts = [-S * 14 // 100 + k * S for k in range(40)]
    fault = [c for c in cuts if 2 * S <= c <= 15 * S]  # every whole window but the first attributed
    attrs = [_attr(c, "cpu_throttle") for c in fault]
    res = score([("fault_cpu", 0, 15 * S)], attrs, 1000.0, expect={"fault_cpu": {"cpu_throttle"}}, cuts=cuts)
    d = res["phases"]["fault_cpu"]
    assert d["windows"] == 14 and d["top1"] == {"cpu_throttle": 13, "none": 1}
    assert d["accuracy"] == round(13 / 14, 4)
    assert d["detection_delay_s"] == 2.96  # the first correct window (2.86) arrived 0.1 s after its cut
    # without the grid the same attributions read as 13 of 15
    assert score([("fault_cpu", 0, 15 * S)], attrs, 1000.0,
                 expect={"fault_cpu": {"cpu_throttle"}})["phases"]["fault_cpu"]["windows"] == 15
