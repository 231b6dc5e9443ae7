"""Variable-length digest entry points (BRB_MD5Batch, BrbSha1_Batch) on the cfg2 shape, beside the
fixed-stride ones: device mode, HIP events around back-to-back calls."""
import sys

import os
import sys as _s
_s.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch

import brb_framework_amd as brb

n, L = int(sys.argv[1]) if len(sys.argv) > 1 else 65536, int(sys.argv[2]) if len(sys.argv) > 2 else 1500
dev = torch.device("cuda:0")
data = torch.randint(0, 256, (n * L + 64,), dtype=torch.uint8, device=dev)
offs = torch.arange(n, dtype=torch.int64, device=dev) * L
lens = torch.full((n,), L, dtype=torch.int32, device=dev)
out = torch.empty((n, 20), dtype=torch.uint8, device=dev)


def t(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


o16 = torch.empty((n, 16), dtype=torch.uint8, device=dev)
cases = {
    "md5 fixed": lambda: brb.md5_batch_fixed(data, L, n, out=o16, async_=True),
    "md5 var": lambda: brb.md5_batch(data, offs, lens, out=o16, async_=True),
    "sha1 fixed": lambda: brb.sha1_batch_fixed(data, L, n, out=out, async_=True),
    "sha1 var": lambda: brb.sha1_batch(data, offs, lens, out=out, async_=True),
}
for k, f in cases.items():
    us = t(f)
    print(f"{k:10s} {us:8.1f} us  {n * L / us / 1e3:7.1f} GB/s")
