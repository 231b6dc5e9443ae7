"""Fixed cost of a K-step timed region (barrier-free, one rank): the headline's cfg2 launch through
the C ABI, K back-to-back launches between torch.cuda.synchronize() on both sides, after a settle
of >= 1 s of the same launches.  Prints, per K, the median wall time, the event time of the K
launches, and wall - events (what the bracket itself costs).  --spin sets hipDeviceScheduleSpin
through the HIP runtime torch loads, before the device is first used.
    python tools/mb/short_region.py [--spin]"""
import ctypes
import math
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import torch  # noqa: E402

if "--spin" in sys.argv:
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    print("hipSetDeviceFlags(spin) ->", hip.hipSetDeviceFlags(ctypes.c_uint(1)), flush=True)

import brb_framework_amd as brb  # noqa: E402
from brb_framework_amd import workload  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
L, n = 1500, 65536
host = workload.gen_records(workload.SEEDS[2], 0, n, L)
bufs = [torch.from_numpy(host).to(dev)]
for _ in range(6):
    bufs.append(bufs[0].clone())
out = torch.empty((n, 16), dtype=torch.uint8, device=dev)
s = torch.cuda.current_stream(dev)
cfn = brb.lib().BRB_MD5BatchFixed
ptrs = [b.data_ptr() for b in bufs]
op = out.data_ptr()
flags = brb.BATCH_DEVICE | brb.BATCH_ASYNC
k_all = 0


def launch():
    global k_all
    rc = cfn(ptrs[k_all % 7], L, n, op, flags, s.cuda_stream)
    k_all += 1
    assert rc == 1


t0 = time.perf_counter()
while time.perf_counter() - t0 < 1.0:
    for _ in range(200):
        launch()
    torch.cuda.synchronize()

for K in (1, 2, 5, 20, 100):
    walls, evs = [], []
    for rep in range(30):
        for _ in range(50):          # keep the clock up between repetitions
            launch()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t = time.perf_counter()
        e0.record(s)
        for _ in range(K):
            launch()
        e1.record(s)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t)
        evs.append(e0.elapsed_time(e1) / 1e3)
    w, e = statistics.median(walls), statistics.median(evs)
    print(f"K {K:4d}  wall {w * 1e6:8.1f} us  events {e * 1e6:8.1f} us  per step wall {w / K * 1e6:6.2f} "
          f"ev {e / K * 1e6:6.2f}  bracket {(w - e) * 1e6:6.1f} us", flush=True)

# enqueue cost of one launch on the host (the GPU is busy, so this is the C-ABI call alone)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(200):
    launch()
dt = (time.perf_counter() - t) / 200
torch.cuda.synchronize()
print(f"host enqueue per launch {dt * 1e6:.2f} us", flush=True)
