"""bench.py's contract on the CPU: the cfg1 line's fields, and the timed region of the GPU lines
(driven here with a stand-in for torch's CUDA events: the order of event records and launches is
what decides which launches the per-launch time covers)."""
import json
import os
import subprocess
import sys
import types

import pytest

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

    cuda = types.SimpleNamespace(Event=Event, synchronize=lambda: clock.log.append("sync"))
    return types.SimpleNamespace(cuda=cuda)


def test_timed_steps_covers_launches_3_to_k():
    """One stream: e0 is recorded right after launch 2 (it fires when launch 2 ends), e1 after
    launch K, so the per-launch time is (launches 3..K) / (K - 2); the first launches' extra time
    (modelled as 50 ms and 20 ms stalls) stays out of it.  Every event is recorded once before the
    synchronize that opens the region (torch creates the HIP event at its first record), so nothing
    but the launches and their event records sits between the two synchronizes."""
    clock = _Clock()
    torch = _fake_torch(clock, 2.0)

    def launch(k, s, j):
        clock.log.append(f"launch{k}")
        clock.t += 2.0 + (50.0 if k == 0 else 20.0 if k == 1 else 0.0)

    bench.MARK = False
    wall, per = bench.timed_steps(launch, 5, ["s0"], lambda: None, lambda x: x, torch)
    assert clock.log == ["event"] * 3 + ["sync", "event", "launch0", "launch1", "event", "launch2", "launch3",
                                         "launch4", "event", "sync"]
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
    region = clock.log[clock.log.index("sync") + 1:-1]
    assert region[0] == "event" and region[-1] == "event" and region.count("event") == 2
    assert abs(per - 2.0e-3) < 1e-12
    clock.log.clear()
    _, per1 = bench.timed_steps(launch, 1, ["s0"], lambda: None, lambda x: x, torch)
    assert clock.log == ["event"] * 3 + ["sync", "event", "launch0", "event", "sync"] and abs(per1 - 2.0e-3) < 1e-12


def test_timed_steps_restores_gc_when_a_launch_raises():
    """the collector is off only inside the region; a launch that raises there must not
    leave it off for the rest of the run (the cfg5 and host-inclusive legs)."""
    import gc

    clock = _Clock()
    torch = _fake_torch(clock, 2.0)

    def launch(k, s, j):
        if k == 2:
            raise RuntimeError("launch failed")
        clock.t += 2.0

    bench.MARK = False
    assert gc.isenabled()
    with pytest.raises(RuntimeError, match="launch failed"):
        bench.timed_steps(launch, 5, ["s0"], lambda: None, lambda x: x, torch)
    assert gc.isenabled()


# ---- roofline.traffic / roofline.compute come only from a PMC pass of the timed kernels ------------
ROCPROF_NAMES = {
    "cfg2_md5": ["void brb_digest::digest_line_kernel<(anonymous namespace)::Md5Alg, 8, true, true>"
                 "(unsigned char const*, unsigned int, unsigned long, unsigned char*)"],
    "cfg4_blowfish": ["void brb_bf::bf_rep_kernel<2, false>(unsigned long const*, unsigned long*, unsigned long)",
                      "void brb_bf::bf_rep_kernel<2, true>(unsigned long const*, unsigned long*, unsigned long)"],
    "f1_rc4": ["void (anonymous namespace)::rc4_crypt_pair_kernel<false>(unsigned char*, unsigned char const*, "
               "unsigned char*, unsigned long const*, unsigned int const*, unsigned long, ...)"],
    "f1_rc4md5": ["void (anonymous namespace)::rc4md5_frame_pair_kernel<false>(unsigned char*, ...)",
                  "void (anonymous namespace)::rc4md5_open_pair_kernel<false>(unsigned char*, ...)"],
    "f4_metadata": ["void (anonymous namespace)::metadata_line_kernel<4, 2, true, false>(unsigned char const*, ...)"],
    "f4_md5seg": ["void (anonymous namespace)::md5_seg_pc_kernel<4, false>(unsigned char const*, ...)"],
}


def _lib_opt():
    from brb_framework_amd import crypto

    def opt(name):
        old = crypto.test_option(name, 0)
        crypto.test_option(name, old)
        return old
    return opt


def test_kernel_id_and_default_selection():
    """kernel_id strips namespaces and arguments; under the library's default test options the timed
    kernels of each line are the product kernels (the wave pairs for RC4, frames, MetaData, segments)."""
    opt = _lib_opt()
    assert bench.kernel_id(ROCPROF_NAMES["cfg2_md5"][0]) == "digest_line_kernel<Md5Alg, 8, true, true>"
    # round 5's five-argument line kernel (and its POOL / LOCK forms) is not the timed kernel any more
    for old in ("digest_line_kernel<Md5Alg, 8, true, true, true>",
                "digest_line_kernel<Md5Alg, 8, true, true, true, true>"):
        assert not bench.kernels_match([old], bench.timed_kernel_patterns("cfg2_md5", opt))
    assert bench.kernel_id("(anonymous namespace)::rc4md5_open_pair_kernel(unsigned char*, ...") == \
        "rc4md5_open_pair_kernel"
    for key, names in ROCPROF_NAMES.items():
        ids = sorted(bench.kernel_id(n) for n in names)
        assert bench.kernels_match(ids, bench.timed_kernel_patterns(key, opt)), (key, ids)
    # the pre-pair RC4 kernel (round 4's stale f1 evidence) does not pass for the pair line
    assert not bench.kernels_match(["rc4_crypt_kernel<true>"], bench.timed_kernel_patterns("f1_rc4", opt))
    # one-to-one: a missing or an extra kernel fails
    assert not bench.kernels_match(["rc4md5_frame_pair_kernel<false>"], bench.timed_kernel_patterns("f1_rc4md5", opt))
    assert not bench.kernels_match([], bench.timed_kernel_patterns("cfg2_md5", opt))


def test_load_pmc_refuses_other_kernels(tmp_path):
    """A PMC entry of another kernel (or one that does not name its kernels) gives no traffic and a
    refused compute block, never numbers; the matching entry is used."""
    opt = _lib_opt()
    det = {"source": "x.txt", "sq_insts_valu": 2.8e7, "sq_waves": 2048.0, "sq_insts_lds": 1e7}
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps({"f1_rc4": 1000, "f1_rc4_detail": dict(det, kernels=["rc4_crypt_kernel<true>"]),
                             "f4_md5seg": 10, "f4_md5seg_detail": det}))
    old = bench.OPT
    bench.OPT = opt
    try:
        for key in ("f1_rc4", "f4_md5seg"):
            t = bench.traffic_fields(str(p), key)
            assert t["traffic"] is None and "not used" in t["traffic_source"]
            c = bench.issue_compute(str(p), key, 1e-4)
            assert set(c) == {"refused"}
        p.write_text(json.dumps({"f1_rc4": 1000, "f1_rc4_detail": dict(det, kernels=["rc4_crypt_pair_kernel<false>"])}))
        assert bench.traffic_fields(str(p), "f1_rc4")["traffic"] == 1000
        c = bench.issue_compute(str(p), "f1_rc4", 1e-4)
        assert c["kernels"] == ["rc4_crypt_pair_kernel<false>"] and c["waves_per_simd"] == 2.0
    finally:
        bench.OPT = old


def test_committed_evidence_compute_matches_timed_kernels():
    """Every line of the newest committed evidence (profiles/r*_evidence/lines.json written with
    kernel identities) carries roofline.compute from the kernels its timed region launched."""
    import glob
    dirs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_evidence", "lines.json")))
    checked = 0
    for path in reversed(dirs):
        lines = json.load(open(path))
        if not any("timed_kernel_ids" in (e.get("timed_region") or {}) for e in lines.values()):
            continue                          # written before the check existed
        for name, e in lines.items():
            t = e.get("timed_region") or {}
            comp = (e["line"].get("roofline") or {}).get("compute")
            if comp and t:
                assert t.get("compute_kernels_match") is True, (path, name, t.get("compute_kernels"),
                                                               t.get("timed_kernel_ids"))
                checked += 1
        break
    if dirs and checked == 0:
        import pytest
        pytest.skip("no committed evidence with kernel identities yet")


def test_warm_up_settles_before_an_explicit_w():
    """An explicit --warmup W runs after an untimed settle of the same launches (>= settle_s; reported
    as bench.SETTLE), and --settle-s 0 leaves exactly W launches (the PMC passes)."""
    import argparse
    n = [0]
    log = []

    def launch(k, s, j):
        n[0] += 1
    torch = types.SimpleNamespace(cuda=types.SimpleNamespace(synchronize=lambda: log.append(n[0])))
    w, k = bench.warm_up(argparse.Namespace(warmup=5, steps=20, settle_s=0.05), launch, ["s0"], torch, lambda x: x)
    assert (w, k) == (5, 20)
    assert bench.SETTLE and bench.SETTLE["launches"] == n[0] - 5 and bench.SETTLE["seconds"] >= 0.05
    n[0] = 0
    w, k = bench.warm_up(argparse.Namespace(warmup=5, steps=20, settle_s=0.0), launch, ["s0"], torch, lambda x: x)
    assert (w, k) == (5, 20) and n[0] == 5 and bench.SETTLE is None
