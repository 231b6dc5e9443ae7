"""Host cost of one device-mode ASYNC BRB_MD5BatchFixed call (bench.py's launch_raw) against the
kernel's own time: is a 20-step timed region fed fast enough by the host?  Prints the host time per
call for bursts of 20 and 2000 calls, and the HIP-event time per launch of 20 back-to-back launches
(a) as bench.py issues them and (b) queued behind a sleep kernel, so that all 20 are enqueued
before the first one runs."""
import sys
import time

import torch

sys.path.insert(0, ".")
import brb_framework_amd as brb  # noqa: E402
from brb_framework_amd import workload  # noqa: E402

n, L = 65536, 1500
dev = torch.device("cuda", 0)
host = workload.gen_records(workload.SEEDS[2], 0, n, L)
bufs = [torch.from_numpy(host).to(dev) for _ in range(7)]
out = torch.empty((n, 16), dtype=torch.uint8, device=dev)
s = torch.cuda.current_stream(dev)
cfn = brb.lib().BRB_MD5BatchFixed
ptrs = [b.data_ptr() for b in bufs]
optr = out.data_ptr()
flags = brb.BATCH_DEVICE | brb.BATCH_ASYNC
cs = s.cuda_stream


def call(k):
    rc = cfn(ptrs[k % 7], L, n, optr, flags, cs)
    if rc != 1:
        raise RuntimeError(brb.lib().BRB_CryptoGPU_LastError().decode())


for k in range(20000):        # settle
    call(k)
torch.cuda.synchronize()
for burst in (20, 2000):
    t0 = time.perf_counter()
    for k in range(burst):
        call(k)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"host enqueue, burst of {burst}: {(t1 - t0) / burst * 1e6:.2f} us per call")
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for mode in ("as bench", "queued behind a sleep", "as bench", "queued behind a sleep"):
    res = []
    for rep in range(15):
        for k in range(3000):     # re-settle
            call(k)
        torch.cuda.synchronize()
        if mode != "as bench":
            torch.cuda._sleep(2_000_000)   # ~1 ms of GPU time while the 20 calls are enqueued
        for k in range(22):
            call(k)
            if k == 1:
                e0.record(s)
        e1.record(s)
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) * 1000 / 20)
    res.sort()
    print(f"{mode:22s}: us per launch over 20: min {res[0]:.2f} p50 {res[len(res)//2]:.2f} max {res[-1]:.2f}")
