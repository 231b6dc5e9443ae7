#!/usr/bin/env python3
"""Host-side latency of what brackets a bench timed region on the MI355X box: torch.cuda.synchronize()
on an idle device, and one small kernel launched through the C ABI + synchronize, under the HIP
runtime's default scheduling and (argv[1] == "spin") hipDeviceScheduleSpin set before the context
exists.  Prints medians in microseconds."""
import ctypes
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if len(sys.argv) > 1 and sys.argv[1] == "spin":
    hip = ctypes.CDLL("libamdhip64.so")
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(1))      # hipDeviceScheduleSpin
    print("hipSetDeviceFlags(spin) rc", rc)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import brb_framework_amd as brb  # noqa: E402

dev = torch.device("cuda", 0)
x = torch.zeros(1 << 16, dtype=torch.uint8, device=dev)
o = torch.zeros((64, 16), dtype=torch.uint8, device=dev)
s = torch.cuda.current_stream()
fn = brb.lib().BRB_MD5BatchFixed
flags = brb.BATCH_DEVICE | brb.BATCH_ASYNC
for _ in range(200):
    fn(x.data_ptr(), 1024, 64, o.data_ptr(), flags, s.cuda_stream)
torch.cuda.synchronize()
idle, one = [], []
for _ in range(2000):
    t = time.perf_counter()
    torch.cuda.synchronize()
    idle.append(time.perf_counter() - t)
for _ in range(2000):
    t = time.perf_counter()
    fn(x.data_ptr(), 1024, 64, o.data_ptr(), flags, s.cuda_stream)
    torch.cuda.synchronize()
    one.append(time.perf_counter() - t)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
gpu = []
for _ in range(200):
    e0.record(s)
    fn(x.data_ptr(), 1024, 64, o.data_ptr(), flags, s.cuda_stream)
    e1.record(s)
    e1.synchronize()
    gpu.append(e0.elapsed_time(e1) * 1e-3)
print(f"mode {sys.argv[1] if len(sys.argv) > 1 else 'default'}: idle synchronize {statistics.median(idle) * 1e6:.1f} us, "
      f"launch + synchronize {statistics.median(one) * 1e6:.1f} us, the kernel by events {statistics.median(gpu) * 1e6:.1f} us")
