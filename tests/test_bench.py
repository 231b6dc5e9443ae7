"""bench.py's contract on the CPU: the cfg1 line's fields, and the timed region of the GPU lines
(driven here with a stand-in for torch's CUDA events: the order of event records and launches is
what decides which launches the per-launch time covers)."""
import json
import os
import subprocess
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

FIELDS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
          "vs_baseline", "dtype", "data", "config"}


def test_cfg1_line_fields():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "1", "--steps", "3",
                          "--warmup", "1"], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert FIELDS <= set(d)
    assert d["steps"] == 3 and d["warmup"] == 1 and d["value"] > 0 and d["higher_is_better"] is True
    assert d["config"]["workload"].startswith("cfg1")


class _Clock:
    def __init__(self):
        self.t = 0.0          # GPU time in ms
        self.log = []


def _fake_torch(clock, kernel_ms):
    class Event:
        def __init__(self, enable_timing=False):
            self.at = None

        def record(self, stream=None):
            self.at = clock.t
            clock.log.append("event")

        def elapsed_time(self, other):
            return other.at - self.at

    cuda = types.SimpleNamespace(Event=Event, synchronize=lambda: None)
    return types.SimpleNamespace(cuda=cuda)


def test_timed_steps_covers_launches_3_to_k():
    """One stream: e0 is recorded right after launch 2 (it fires when launch 2 ends), e1 after
    launch K, so the per-launch time is (launches 3..K) / (K - 2); the first launches' extra time
    (modelled as 50 ms and 20 ms stalls) stays out of it."""
    clock = _Clock()
    torch = _fake_torch(clock, 2.0)

    def launch(k, s, j):
        clock.log.append(f"launch{k}")
        clock.t += 2.0 + (50.0 if k == 0 else 20.0 if k == 1 else 0.0)

    bench.MARK = False
    wall, per = bench.timed_steps(launch, 5, ["s0"], lambda: None, lambda x: x, torch)
    assert clock.log == ["event", "launch0", "launch1", "event", "launch2", "launch3", "launch4", "event"]
    assert abs(per - 2.0e-3) < 1e-12          # seconds per launch
    assert abs(bench.LAST_ALL_K_S - (5 * 2.0 + 70.0) / 5 / 1e3) < 1e-12   # all K, the stalls included
    assert wall >= 0


def test_timed_steps_multi_stream_brackets_all():
    """Several streams (or K < 3): the events bracket every launch and the time is divided by K."""
    clock = _Clock()
    torch = _fake_torch(clock, 2.0)

    def launch(k, s, j):
        clock.log.append(f"launch{k}")
        clock.t += 2.0

    bench.MARK = False
    _, per = bench.timed_steps(launch, 4, ["s0", "s1"], lambda: None, lambda x: x, torch)
    assert clock.log[0] == "event" and clock.log[-1] == "event"
    assert abs(per - 2.0e-3) < 1e-12
    clock.log.clear()
    _, per1 = bench.timed_steps(launch, 1, ["s0"], lambda: None, lambda x: x, torch)
    assert clock.log == ["event", "launch0", "event"] and abs(per1 - 2.0e-3) < 1e-12
