"""GPU parity at the edges of the digest and Blowfish batch paths (SURVEY §8(a), §7 edge cases):
empty batches, records on both sides of the line kernel's 1 MiB limit (digest_line.h
`line_supported`), and batches whose bytes run past 4 GiB (64-bit record addressing in the buffer
descriptors).  The oracle, or hashlib where the oracle would take minutes, is the checker.
"""
import hashlib

import numpy as np
import pytest

from brb_framework_amd import workload

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev(brb):
    import torch
    assert torch.cuda.is_available(), "no HIP device visible to torch"
    assert brb.gpu_available(), brb.lib().BRB_CryptoGPU_LastError()
    return torch


def test_empty_batches(brb, torch_dev):
    """n = 0 is a completed call (return code 1) that touches nothing, NULL pointers included
    (the transform hook's "nothing to do"), in host and device mode."""
    lib = brb.lib()
    for fn in (lib.BRB_MD5BatchFixed, lib.BrbSha1_BatchFixed):
        assert fn(None, 1500, 0, None, 0, None) == 1
        assert fn(None, 1500, 0, None, brb.BATCH_DEVICE, None) == 1
    for fn in (lib.BRB_MD5Batch, lib.BrbSha1_Batch):
        assert fn(None, None, None, 0, None, 0, None) == 1
    d = torch_dev.zeros(64, dtype=torch_dev.uint8, device="cuda")
    out = torch_dev.full((1, 16), 0xA5, dtype=torch_dev.uint8, device="cuda")
    brb.md5_batch_fixed(d, 64, 0, out=out)
    assert int(out.min()) == 0xA5 and int(out.max()) == 0xA5          # untouched
    assert brb.md5_batch_fixed(np.zeros(0, np.uint8), 1500, 0).shape == (0, 16)
    ctx = brb.blowfish_init(b"TESTKEY")
    w = torch_dev.arange(8, dtype=torch_dev.int64, device="cuda")
    brb.blowfish_encrypt_batch(ctx, w, n_blocks=0)
    assert w.cpu().tolist() == list(range(8))


@pytest.mark.parametrize("rec_len", [
    1 << 20,              # the longest record the line-staged kernel takes
    (1 << 20) + 4,        # 4-byte multiple past it: record-relative stages (digest_dma.h)
    (1 << 20) + 1,        # odd length: record-relative stages, tail of 1 byte
    (2 << 20) + 60,       # t = 60: two padding blocks
])
def test_records_around_line_limit(brb, orc, torch_dev, rec_len):
    n = 130                                        # two full 64-record groups and a partial one
    data = workload.gen_records(0x5EED0021, 0, n, rec_len)
    want5 = orc.md5_batch_fixed(data, rec_len, n, threads=16)
    d = torch_dev.from_numpy(data).cuda()
    assert np.array_equal(brb.md5_batch_fixed(d, rec_len, n).cpu().numpy(), want5)
    assert np.array_equal(brb.md5_batch_fixed(data, rec_len, n), want5)           # host mode, chunked
    if rec_len != 1 << 20:
        want1 = orc.sha1_batch_fixed(data, rec_len, n, threads=16)
        assert np.array_equal(brb.sha1_batch_fixed(d, rec_len, n).cpu().numpy(), want1)


@pytest.mark.parametrize("rec_len", [65540, 65538])
def test_batch_past_4gib(brb, torch_dev, rec_len):
    """65 600 records of ~64 KiB = 4.3 GB: record bases past 2^32 in the line kernel (65 540 B) and
    the record-relative one (65 538 B).  Device-mode digests of every record equal the host-mode
    (chunked pipeline) ones; 96 records, the ones around the 4 GiB boundary and the last included,
    equal hashlib."""
    torch = torch_dev
    n = 65600
    nbytes = n * rec_len
    assert nbytes > 1 << 32
    g = torch.Generator(device="cuda").manual_seed(rec_len)
    d = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda", generator=g)
    got = brb.md5_batch_fixed(d, rec_len, n).cpu().numpy()
    got1 = brb.sha1_batch_fixed(d, rec_len, n).cpu().numpy()
    host = d.cpu().numpy()
    del d
    torch.cuda.empty_cache()
    assert np.array_equal(brb.md5_batch_fixed(host, rec_len, n), got)
    edge = (1 << 32) // rec_len
    rng = np.random.default_rng(rec_len)
    picks = sorted(set(rng.integers(0, n, 88).tolist()) | {0, edge - 1, edge, edge + 1, n - 64, n - 2, n - 1})
    for r in picks:
        rec = host[r * rec_len:(r + 1) * rec_len].tobytes()
        assert got[r].tobytes() == hashlib.md5(rec).digest(), f"md5 record {r}"
        assert got1[r].tobytes() == hashlib.sha1(rec).digest(), f"sha1 record {r}"


def test_random_record_shapes(brb, orc, torch_dev):
    """A seeded sweep of 48 record shapes: lengths from 1 B to 12 KiB (so their residues mod 128,
    which set the line kernel's window shifts, and mod 4, which pick the kernel, vary), base offsets
    0..15 and batch sizes around the 64-record group; device mode against the oracle on every
    record, MD5 and SHA-1."""
    rng = np.random.default_rng(0x5EED0031)
    for case in range(48):
        rec_len = int(rng.integers(1, 12289)) if case % 3 else int(rng.integers(65, 400))
        n = int(rng.choice([1, 63, 64, 65, 127, 129, 300]))
        off = int(rng.integers(0, 16))
        data = workload.gen_records(0x5EED0040 + case, 0, n, rec_len)
        d = torch_dev.zeros(off + data.size + 8, dtype=torch_dev.uint8, device="cuda")
        d[off:off + data.size] = torch_dev.from_numpy(data).cuda()
        view = d[off:off + data.size]
        assert np.array_equal(brb.md5_batch_fixed(view, rec_len, n).cpu().numpy(),
                              orc.md5_batch_fixed(data, rec_len, n, threads=8)), (case, rec_len, n, off)
        assert np.array_equal(brb.sha1_batch_fixed(view, rec_len, n).cpu().numpy(),
                              orc.sha1_batch_fixed(data, rec_len, n, threads=8)), (case, rec_len, n, off)
