#!/usr/bin/env python3
"""Host-mode (PCIe-inclusive) rates vs chunk size: for each setting a fresh process
(chunk sizes set through the test options host_digest_chunk_mib / host_chunk_mib) times cfg2 and cfg3 digests and the cfg4 Blowfish round
trip from pageable and page-locked host memory.

Usage: python tools/host_sweep.py [digest_chunk_MiB,blowfish_chunk_MiB ...]   (default: 32,16)"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch

    import brb_framework_amd as brb
    from brb_framework_amd import workload

    def rate(call, nbytes, reps):
        call()
        t = time.perf_counter()
        for _ in range(reps):
            call()
        dt = (time.perf_counter() - t) / reps
        return round(nbytes / dt / 1e9, 2)

    d_mib, b_mib = (int(x) for x in os.environ["HOST_SWEEP_CHILD"].split(","))
    brb.test_option("host_digest_chunk_mib", d_mib)
    brb.test_option("host_chunk_mib", b_mib)
    res = {"digest_chunk_mib": d_mib, "chunk_mib": b_mib}
    for c in (2, 3):
        cfg = workload.CONFIGS[c]
        n, L = cfg["records"], cfg["rec_len"]
        host = workload.gen_records(workload.SEEDS[c], 0, n, L)
        out = np.empty((n, 16), np.uint8)
        pin = torch.from_numpy(host).pin_memory().numpy()
        res[f"cfg{c}_pageable_GBs"] = rate(lambda: brb.md5_batch_fixed(host, L, n, out=out), host.nbytes, 8)
        res[f"cfg{c}_pinned_GBs"] = rate(lambda: brb.md5_batch_fixed(pin, L, n, out=out), host.nbytes, 8)
    w = workload.gen_words(workload.SEEDS[4], 1 << 27)
    ctx = brb.blowfish_init(workload.CFG4_KEY)

    def trip(b):
        brb.blowfish_encrypt_batch(ctx, b)
        brb.blowfish_decrypt_batch(ctx, b)

    res["cfg4_pageable_GBs_plaintext"] = rate(lambda: trip(w), w.nbytes, 2)
    pw = torch.from_numpy(w.view(np.int64)).pin_memory().numpy().view(np.uint64)
    res["cfg4_pinned_GBs_plaintext"] = rate(lambda: trip(pw), w.nbytes, 2)
    print(json.dumps(res), flush=True)


def main():
    if os.environ.get("HOST_SWEEP_CHILD"):
        child()
        return
    settings = sys.argv[1:] or ["32,16"]
    for st in settings:
        d, b = (int(x) for x in st.split(","))
        env = dict(os.environ, HOST_SWEEP_CHILD=f"{d},{b}")
        subprocess.run([sys.executable, __file__], env=env, check=True, timeout=300)


if __name__ == "__main__":
    main()
