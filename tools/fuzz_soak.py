"""Soak run of tests/test_gpu_fuzz.py: every fuzz test over fresh seeds until a time budget runs out,
printing a progress line per round.  Stops at the first mismatch (the seed is in the message).
    python tools/fuzz_soak.py [--scale=k] [seconds] [first_seed] [batcher]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

for a in list(sys.argv[1:]):                  # --scale k: batch sizes x k (BRB_FUZZ_SCALE)
    if a.startswith("--scale="):
        os.environ["BRB_FUZZ_SCALE"] = a.split("=", 1)[1]
        sys.argv.remove(a)

import torch  # noqa: E402

import brb_framework_amd as brb  # noqa: E402
import oracle  # noqa: E402
import test_batcher as B  # noqa: E402
import test_gpu_fuzz as F  # noqa: E402

budget = float(sys.argv[1]) if len(sys.argv) > 1 else 240.0
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
batcher = len(sys.argv) > 3 and sys.argv[3] == "batcher"     # the event loop of test_batcher.py instead
brb.lib()
oracle.lib()
assert torch.cuda.is_available() and brb.gpu_available()
t0 = time.time()
cases = 0
while batcher and time.time() - t0 < budget:
    for algo in (1, 2):
        for zc in (False, True):
            for pl in (False, True):
                B._event_loop(brb, oracle, algo, zc, pl, seed=seed, rounds=4)
    cases += 8
    print(f"batcher seed {seed} ok  ({cases} event loops of 4 rounds, {time.time() - t0:.0f} s)", flush=True)
    seed += 1
while not batcher and time.time() - t0 < budget:
    F.test_fuzz_fixed_stride(brb, oracle, torch, seed)
    F.test_fuzz_variable_length(brb, oracle, torch, seed)
    for sl in (0, 1, 2):
        F.test_fuzz_segments(brb, torch, seed, sl)
    F.test_fuzz_rc4(brb, oracle, torch, seed)
    F.test_fuzz_rc4md5_frame_open(brb, oracle, torch, seed)
    F.test_fuzz_base64(brb, oracle, torch, seed)
    F.test_fuzz_blowfish(brb, oracle, torch, seed)
    F.test_fuzz_host_mode(brb, oracle, torch, seed)
    cases += 10
    print(f"seed {seed} ok  ({cases} cases, {time.time() - t0:.0f} s)", flush=True)
    seed += 1
print(f"soak{' (batcher)' if batcher else ''}: {cases} cases over seeds up to {seed - 1}, no mismatch", flush=True)
