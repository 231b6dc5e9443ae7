#!/usr/bin/env python3
"""Where a wave of the line-staged segment kernel spends its cycles (in-kernel s_memtime stamps).

Run with the diagnostic library (make -C brb_framework_amd diag):
    BRB_CRYPTO_LIB=brb_framework_amd/build-diag/libbrb_crypto_gpu.so python3 tools/seg_probe.py [--pc]
(--pc: the producer / consumer kernel, seg_line 2: each wave's waits for the other and the DMA)
The diagnostic md5_seg_line_kernel writes, instead of digests, per group: into record 64g's slot the
cycles spent in the top-of-line DMA wait, the window read, the stage (cursor + DMA issue) and the
word emission; into record 64g+1's slot the pumps (compressions), the group's total and its line
count K.  Shape: the md5seg bench (65 536 records x 4 segments of 375 B inside 1 664-byte packs).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import brb_framework_amd as brb
    from brb_framework_amd import workload
    assert "build-diag" in brb.crypto.LIB_PATH, "set BRB_CRYPTO_LIB to the diagnostic build"
    n, K, Q = 65536, 4, 375
    stride = 64 + K * (24 + Q + 1)
    pool = workload.gen_records(0x5EED0002, 0, 1, n * stride + 64)
    offs = (np.arange(n, dtype=np.uint64)[:, None] * stride + 64 + 24
            + np.arange(K, dtype=np.uint64)[None, :] * (25 + Q)).reshape(-1).astype(np.uint64)
    lens = np.full(n * K, Q, np.uint32)
    first = (np.arange(n + 1, dtype=np.uint64) * K).astype(np.uint64)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()   # noqa: E731
    d, o, ln, fi = dev(pool), dev(offs), dev(lens), dev(first)
    pc = "--pc" in sys.argv
    with brb.TestOption("seg_line", 2 if pc else 1):
        for _ in range(20):
            out = brb.md5_batch_segments(d, o, ln, fi)
    torch.cuda.synchronize()
    v = out.cpu().numpy().reshape(-1).view(np.uint32).reshape(n, 4)
    a, b = v[0::64], v[1::64]
    if pc:      # producer: waits for the consumer, DMA waits, total, K; consumer: waits, total, K
        pt, ct = a[:, 2].astype(np.float64), b[:, 1].astype(np.float64)
        print(f"groups {len(pt)}, K {int(np.median(a[:, 3]))}; producer total {np.median(pt):.0f} cycles: "
              f"waits for the consumer {np.median(a[:, 0] / pt):.3f}, for its DMA {np.median(a[:, 1] / pt):.3f}; "
              f"consumer total {np.median(ct):.0f}: waits for the producer {np.median(b[:, 0] / ct):.3f}")
        return
    parts = {"wait": a[:, 0], "window": a[:, 1], "stage": a[:, 2], "emit": a[:, 3], "pump": b[:, 0]}
    total = b[:, 1].astype(np.float64)
    print(f"groups {len(total)}, lines per group (median) {int(np.median(b[:, 2]))}, "
          f"total cycles per group: median {np.median(total):.0f}")
    for k, x in parts.items():
        print(f"  {k:7s} median {np.median(x):9.0f} cycles  ({np.median(x / total):.3f} of the group)")
    rest = total - sum(x.astype(np.float64) for x in parts.values())
    print(f"  {'rest':7s} median {np.median(rest):9.0f} cycles  ({np.median(rest / total):.3f})")


if __name__ == "__main__":
    main()
