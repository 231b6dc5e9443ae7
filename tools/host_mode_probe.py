#!/usr/bin/env python3
"""Host-mode call timeline (run under rocprofv3 --kernel-trace --memory-copy-trace --stats):
cfg3-shaped MD5 batch from pageable then from page-locked (torch pin_memory) input, and the cfg4
Blowfish round trip, a few calls each, so the copies and kernels of both can be compared."""
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import numpy as np  # noqa: E402
import torch  # noqa: E402

import brb_framework_amd as brb  # noqa: E402
from brb_framework_amd import workload  # noqa: E402

n, L = 1 << 20, 64
host = workload.gen_records(workload.SEEDS[3], 0, n, L)
out = np.empty((n, 16), np.uint8)
pin = torch.from_numpy(host).pin_memory().numpy()
for name, buf in (("pageable", host), ("pinned", pin), ("pageable", host), ("pinned", pin)):
    brb.md5_batch_fixed(buf, L, n, out=out)
    t = time.perf_counter()
    for _ in range(5):
        brb.md5_batch_fixed(buf, L, n, out=out)
    print(name, "%.3f ms" % ((time.perf_counter() - t) / 5 * 1e3), flush=True)
