"""Concurrency soak: several host threads call the batch entry points at once for a time budget, each
on its own HIP stream (device mode, sync and async) or through host mode, and check every result
against oracle digests computed up front.  The library keeps per-thread workspaces, pipes and fault
words; this is the many-threads shape of a receive loop's workers.
    python tools/thread_soak.py [--devices=k] [seconds] [threads]"""
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import brb_framework_amd as brb  # noqa: E402
import oracle  # noqa: E402

parts = 0
for a in list(sys.argv[1:]):                  # --devices=k: add all-devices calls forced into k parts
    if a.startswith("--devices="):
        parts = int(a.split("=", 1)[1])
        sys.argv.remove(a)
budget = float(sys.argv[1]) if len(sys.argv) > 1 else 120.0
nthreads = int(sys.argv[2]) if len(sys.argv) > 2 else 8
assert torch.cuda.is_available() and brb.gpu_available()
if parts:
    brb.test_option("devices", parts)
rng = np.random.default_rng(0x50AC)
sets = []
for i in range(6):                                   # (data, offsets, lengths, md5, sha1) per set
    n = int(rng.integers(500, 20000))
    lens = rng.integers(0, 3000, n).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64) + 3)[:-1]]).astype(np.uint64)
    data = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 8, dtype=np.uint8)
    sets.append((data, offs, lens, oracle.md5_batch(data, offs, lens, threads=8),
                 oracle.sha1_batch(data, offs, lens, threads=8)))
fixed = rng.integers(0, 256, 1500 * 30000, dtype=np.uint8)
fixed_md5 = oracle.md5_batch_fixed(fixed, 1500, 30000, threads=8)
bf_key = b"thread-soak-key"
bf_words = rng.integers(0, 2**63, 2 * 50000, dtype=np.int64)
dev_sets = [tuple(torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (d, o.view(np.int64), ln.view(np.int32)))
            for d, o, ln, _, _ in sets]
dev_fixed = torch.from_numpy(fixed).cuda()
torch.cuda.synchronize()
errors, counts, stop = [], [0] * nthreads, time.time() + budget


def worker(t):
    r = np.random.default_rng(1000 + t)
    stream = torch.cuda.Stream()
    ctx = brb.blowfish_init(bf_key)
    try:
        while time.time() < stop and not errors:
            kind = int(r.integers(0, 8 if parts else 6))
            i = int(r.integers(0, len(sets)))
            data, offs, lens, want5, want1 = sets[i]
            if kind == 0:                            # host mode
                assert np.array_equal(brb.md5_batch(data, offs, lens), want5), ("host md5", t, i)
            elif kind == 1:
                assert np.array_equal(brb.sha1_batch(data, offs, lens), want1), ("host sha1", t, i)
            elif kind == 2:                          # device mode on this thread's stream
                d, o, ln = dev_sets[i]
                with torch.cuda.stream(stream):
                    got = brb.md5_batch(d, o, ln, stream=stream)
                stream.synchronize()
                assert np.array_equal(got.cpu().numpy(), want5), ("device md5", t, i)
            elif kind == 3:                          # device mode, async, then the thread's fault check
                with torch.cuda.stream(stream):
                    got = brb.md5_batch_fixed(dev_fixed, 1500, 30000, stream=stream, async_=True)
                stream.synchronize()
                brb.async_fault_check()
                assert np.array_equal(got.cpu().numpy(), fixed_md5), ("async fixed", t)
            elif kind == 4:                          # Blowfish round trip in host mode
                w = bf_words.copy()
                brb.blowfish_encrypt_batch(ctx, w)
                brb.blowfish_decrypt_batch(ctx, w)
                assert np.array_equal(w, bf_words), ("blowfish", t)
            elif kind == 5:                          # host-mode fixed stride
                assert np.array_equal(brb.md5_batch_fixed(fixed, 1500, 30000), fixed_md5), ("host fixed", t)
            elif kind == 6:                          # all-devices split (forced parts)
                got = brb.md5_batch(data, offs, lens, all_devices=True)
                assert np.array_equal(got, want5), ("all-devices md5", t, i)
            else:
                got = brb.md5_batch_fixed(fixed, 1500, 30000, all_devices=True)
                assert np.array_equal(got, fixed_md5), ("all-devices fixed", t)
            counts[t] += 1
    except Exception as e:                           # noqa: BLE001 -- reported below, ends the soak
        errors.append(repr(e))


threads = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
for th in threads:
    th.start()
t0 = time.time()
while any(th.is_alive() for th in threads):
    time.sleep(20)
    print(f"{time.time() - t0:.0f} s: {sum(counts)} calls checked, {len(errors)} errors", flush=True)
for th in threads:
    th.join()
if errors:
    print("FAILED:", errors[0], flush=True)
    sys.exit(1)
print(f"thread soak: {nthreads} threads, {sum(counts)} calls checked in {budget:.0f} s, no mismatch", flush=True)
