"""bench.py's own warm_up (explicit W = 5, with its settle) and timed_steps (K = 20) on the cfg2
launch, repeated: where a 20-step region's wall time goes beyond its kernels.  For each region the
host times of the first launch call, the last launch's return and the region's end are kept.
    python tools/mb/short_region2.py [reps]"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import brb_framework_amd as brb  # noqa: E402
from brb_framework_amd import workload  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
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
marks = []


def launch(k, st, j=0):
    if k == 0:
        marks.append(time.perf_counter())
    rc = cfn(ptrs[k % 7], L, n, op, flags, st.cuda_stream)
    if rc != 1:
        raise RuntimeError("launch failed")
    if k == 19:
        marks.append(time.perf_counter())


def same(x):
    return x


args = argparse.Namespace(warmup=5, steps=20)
rows = []
for r in range(reps):
    w, k = bench.warm_up(args, launch, [s], torch, same)
    marks.clear()
    t = time.perf_counter()
    wall, ev = bench.timed_steps(launch, k, [s], lambda: None, same, torch)
    t_end = time.perf_counter()
    rows.append((wall, ev, bench.LAST_ALL_K_S, marks[0] - t, marks[1] - marks[0], t_end - marks[1]))
    print(f"rep {r:2d} wall/step {wall / 20 * 1e6:6.2f} us  ev {ev * 1e6:6.2f}  all_k {bench.LAST_ALL_K_S * 1e6:6.2f}  "
          f"to first launch {rows[-1][3] * 1e6:6.1f} us  launches {rows[-1][4] * 1e6:6.1f} us  "
          f"after last {rows[-1][5] * 1e6:6.1f} us", flush=True)
print("median wall/step %.2f us, all_k %.2f us" % (statistics.median(r[0] for r in rows) / 20 * 1e6,
                                                   statistics.median(r[2] for r in rows) * 1e6))
