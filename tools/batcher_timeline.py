#!/usr/bin/env python3
"""Where a transform-batcher round's time goes, from one
rocprofv3 --kernel-trace --memory-copy-trace run of tools/batcher_bench (tools/gpu_batcher_trace.sh).

A round is one rc4md5_open_kernel (the READ side) and one rc4md5_frame_kernel (the WRITE side) plus
the round's metadata copies.  For the rounds after warm-up it prints, per round (medians):
  period      start of one round's open kernel to the next round's
  open / frame  kernel durations (zero-copy: the kernels read and write host memory over PCIe)
  overlap     time both kernels ran at once
  copies      memory-copy busy time inside the period (H2D of the round's metadata, D2H in copy mode)
  gpu_idle    time inside the period with neither a kernel nor a copy on the GPU: the host's share
              (submit loop, callbacks, FlushAsync bookkeeping) that nothing on the GPU hid
Usage: tools/batcher_timeline.py <rocprofv3 output dir> [skip_rounds=5]
"""
import csv
import glob
import statistics
import sys


def rows(d, name):
    out = []
    for p in glob.glob(f"{d}/**/*{name}.csv", recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def busy(iv, lo, hi):
    """Length of the union of intervals clipped to [lo, hi)."""
    t, cur = 0, lo
    for a, b in sorted(iv):
        a, b = max(a, cur), min(b, hi)
        if b > a:
            t += b - a
            cur = b
    return t


def main():
    d = sys.argv[1]
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows(d, "kernel_trace")]
    cs = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows(d, "memory_copy_trace")]
    opens = sorted(k for k in ks if "rc4md5_open" in k[2])
    frames = sorted(k for k in ks if "rc4md5_frame" in k[2])
    kern = [(a, b) for a, b, _ in ks]
    per = []
    for i in range(skip, min(len(opens), len(frames)) - 1):
        lo, hi = opens[i][0], opens[i + 1][0]
        o, fr = opens[i], frames[i]
        ov = max(0, min(o[1], fr[1]) - max(o[0], fr[0]))
        cp = busy(cs, lo, hi)
        anyb = busy(kern + cs, lo, hi)
        per.append(dict(period=hi - lo, open=o[1] - o[0], frame=fr[1] - fr[0], overlap=ov, copies=cp,
                        gpu_idle=(hi - lo) - anyb))
    if not per:
        print("no rounds found")
        return
    med = {k: statistics.median(p[k] for p in per) / 1e3 for k in per[0]}
    print(f"{len(per)} rounds (after {skip}); medians in us: " +
          ", ".join(f"{k} {v:.1f}" for k, v in med.items()))


if __name__ == "__main__":
    main()
