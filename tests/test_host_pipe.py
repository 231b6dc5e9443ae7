"""Host-mode batches (host_pipe.hip) and the multi-device runtime, against the oracle.

Host mode copies straight from the caller's memory in 16 MiB chunks, overlapping the H2D copy of one
chunk with the kernel on the previous one and (Blowfish) the D2H copy of an earlier one.  These tests
cut batches so that chunk boundaries fall inside records and the last chunk is short, with pageable
(numpy) and page-locked (torch pin_memory) buffers, and run the BRB_BATCH_ALL_DEVICES split (contiguous
record ranges over every visible device; one range on a one-GPU box).  Every result is compared
with the oracle bit for bit.
"""
import ctypes
import threading

import numpy as np
import pytest

from brb_framework_amd import workload

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu(brb):
    assert brb.gpu_available(), brb.lib().BRB_CryptoGPU_LastError()
    return brb


def pinned_copy(a):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(a)).pin_memory()
    return t, t.numpy()


@pytest.mark.parametrize("n,rec_len", [
    (30_000, 1500),      # 45 MB: three chunks, chunk edges at whole records (line-staged kernel)
    (23_456, 1501),      # record-relative kernel, ragged last chunk
    (400_000, 64),       # 64-byte records: 25.6 MB, two chunks
    (12, 3_000_000),     # 3 MB records: five per chunk
])
def test_fixed_digests_chunked(gpu, orc, n, rec_len):
    data = workload.gen_records(0x5EED0007, 0, n, rec_len)
    want5 = orc.md5_batch_fixed(data, rec_len, n, threads=16)
    assert np.array_equal(gpu.md5_batch_fixed(data, rec_len, n), want5)
    _, pin = pinned_copy(data)
    assert np.array_equal(gpu.md5_batch_fixed(pin, rec_len, n), want5)
    if rec_len != 64:
        assert np.array_equal(gpu.sha1_batch_fixed(data, rec_len, n), orc.sha1_batch_fixed(data, rec_len, n, threads=16))


@pytest.mark.parametrize("pinned", [False, True])
def test_blowfish_chunked_round_trip(gpu, orc, pinned):
    """48 MiB + 7 blocks: three full 16 MiB chunks and a short one; encrypt vs the oracle, then
    decrypt back to the plaintext (D2H of earlier chunks overlaps H2D of later ones)."""
    nb = 3 * (1 << 20) + 7
    w = workload.gen_words(workload.SEEDS[4], 2 * nb)
    ctx = gpu.blowfish_init(workload.CFG4_KEY)
    want = orc.bf_ecb(orc.bf_init(workload.CFG4_KEY), w.copy(), threads=16)
    if pinned:
        _keep, buf = pinned_copy(w)
    else:
        buf = w.copy()
    gpu.blowfish_encrypt_batch(ctx, buf)
    assert np.array_equal(buf, want)
    gpu.blowfish_decrypt_batch(ctx, buf)
    assert np.array_equal(buf, w)


def test_all_devices_digests(gpu, orc):
    n, L = 70_001, 1500
    data = workload.gen_records(0x5EED0008, 0, n, L)
    assert np.array_equal(gpu.md5_batch_fixed(data, L, n, all_devices=True), orc.md5_batch_fixed(data, L, n, threads=16))
    assert np.array_equal(gpu.sha1_batch_fixed(data, L, n, all_devices=True), orc.sha1_batch_fixed(data, L, n, threads=16))
    # variable-length records (BRB_MD5Batch / BrbSha1_Batch): ranges of records, each with its span
    rng = np.random.default_rng(5)
    m = 5000
    lens = rng.integers(0, 3000, m).astype(np.uint32)
    offs = rng.integers(0, data.size - 3000, m).astype(np.uint64)
    want5 = orc.md5_batch(data, offs, lens)
    assert np.array_equal(gpu.md5_batch(data, offs, lens, all_devices=True), want5)
    assert np.array_equal(gpu.sha1_batch(data, offs, lens, all_devices=True), orc.sha1_batch(data, offs, lens))


def test_all_devices_blowfish(gpu, orc):
    nb = 100_003
    w = workload.gen_words(workload.SEEDS[4], 2 * nb)
    ctx = gpu.blowfish_init(b"TESTKEY")
    buf = w.copy()
    gpu.blowfish_encrypt_batch(ctx, buf, all_devices=True)
    assert np.array_equal(buf, orc.bf_ecb(orc.bf_init(b"TESTKEY"), w.copy(), threads=16))
    gpu.blowfish_decrypt_batch(ctx, buf, all_devices=True)
    assert np.array_equal(buf, w)


def test_all_devices_refuses_device_pointers(gpu):
    import torch
    d = torch.zeros(1500 * 4, dtype=torch.uint8, device="cuda")
    out = torch.zeros((4, 16), dtype=torch.uint8, device="cuda")
    L = gpu.lib()
    assert L.BRB_MD5BatchFixed(d.data_ptr(), 1500, 4, out.data_ptr(), gpu.BATCH_DEVICE | gpu.BATCH_ALL_DEVICES, None) == -1
    assert b"ALL_DEVICES" in L.BRB_CryptoGPU_LastError()


def test_device_runtime(gpu, orc):
    L = gpu.lib()
    n = L.BRB_CryptoGPU_DeviceCount()
    assert n >= 1 and gpu.device_count() == n
    assert L.BRB_CryptoGPU_SetDevice(n) == -1 and L.BRB_CryptoGPU_SetDevice(-1) == -1
    for g in range(n):
        assert L.BRB_CryptoGPU_SetDevice(g) == 1 and L.BRB_CryptoGPU_GetDevice() == g
    assert L.BRB_CryptoGPU_SetDevice(0) == 1
    data = workload.gen_records(0x5EED0009, 0, 1000, 700)
    want = orc.md5_batch_fixed(data, 700, 1000)
    assert np.array_equal(gpu.md5_batch_fixed(data, 700, 1000), want)
    L.BRB_CryptoGPU_ThreadCleanup()            # frees this thread's scratch; the next call rebuilds it
    assert np.array_equal(gpu.md5_batch_fixed(data, 700, 1000), want)


def test_event_threads_with_cleanup(gpu, orc):
    """Event threads that come and go: each runs host-mode batches (chunked and all-devices) and
    frees its scratch before it ends; results stay bit-exact."""
    n, L = 13_000, 1500
    data = workload.gen_records(0x5EED000A, 0, n, L)
    want = orc.md5_batch_fixed(data, L, n, threads=16)
    errs = []

    def run(k):
        try:
            for _ in range(3):
                assert np.array_equal(gpu.md5_batch_fixed(data, L, n, all_devices=bool(k & 1)), want)
            gpu.lib().BRB_CryptoGPU_ThreadCleanup()
        except Exception as e:       # noqa: BLE001 -- reported below
            errs.append(repr(e))

    ts = [threading.Thread(target=run, args=(k,)) for k in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs


def test_small_host_batches_stay_exact(gpu, orc):
    """A kqueue round often hands over a few buffers: a single chunk each."""
    for n, L in ((1, 1), (1, 1500), (3, 64), (64, 1500)):
        data = workload.gen_records(0x5EED000B, 0, n, L)
        assert np.array_equal(gpu.md5_batch_fixed(data, L, n), orc.md5_batch_fixed(data, L, n))
    w = workload.gen_words(1, 2)
    ctx = gpu.blowfish_init(b"k")
    buf = w.copy()
    gpu.blowfish_encrypt_batch(ctx, buf)
    assert np.array_equal(buf, orc.bf_ecb(orc.bf_init(b"k"), w.copy()))
    assert ctypes.sizeof(gpu.BRB_BLOWFISH_CTX) == 8336
