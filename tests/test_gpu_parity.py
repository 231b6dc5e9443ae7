"""GPU parity: the HIP batch kernels (through the C ABI) against the CPU oracle, bit for bit.

Small cases run the oracle on every record; full BASELINE sizes are checked against the oracle on
all records where it finishes in seconds (cfg2, cfg3, cfg4's 1 GiB, cfg5's 1 Mi-record shard) plus
size-independent properties (cfg4: exact decrypt(encrypt(x)) == x).
"""
import hashlib

import numpy as np
import pytest

from brb_framework_amd import workload

pytestmark = pytest.mark.gpu

EDGE = [0, 1, 3, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 129, 1500, 16384, 65535, 65536, 65537]


@pytest.fixture(scope="module")
def torch_dev(brb):
    import torch
    assert torch.cuda.is_available(), "no HIP device visible to torch"
    assert brb.gpu_available(), brb.lib().BRB_CryptoGPU_LastError()
    return torch


def to_dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("rec_len", EDGE)
def test_md5_sha1_fixed_edge_lengths(brb, orc, torch_dev, rec_len):
    n = 300 if rec_len <= 16384 else 20
    data = workload.gen_records(0x5EED0001, 0, n, rec_len)
    want5 = orc.md5_batch_fixed(data, rec_len, n, threads=4)
    want1 = orc.sha1_batch_fixed(data, rec_len, n, threads=4)
    # device mode
    d = to_dev(torch_dev, data) if data.size else torch_dev.zeros(1, dtype=torch_dev.uint8, device="cuda")
    assert np.array_equal(brb.md5_batch_fixed(d, rec_len, n).cpu().numpy(), want5)
    assert np.array_equal(brb.sha1_batch_fixed(d, rec_len, n).cpu().numpy(), want1)
    # host mode
    assert np.array_equal(brb.md5_batch_fixed(data, rec_len, n), want5)
    assert np.array_equal(brb.sha1_batch_fixed(data, rec_len, n), want1)


def test_golden_edge_digests(brb, torch_dev, golden):
    g = golden["digests"]
    for e in g["edge"]:
        rec = workload.gen_records(g["generator_seed"], e["record"], 1, e["len"])
        buf = rec if rec.size else np.zeros(1, np.uint8)
        assert brb.md5_batch_fixed(buf, e["len"], 1)[0].tobytes().hex() == e["md5"]
        assert brb.sha1_batch_fixed(buf, e["len"], 1)[0].tobytes().hex() == e["sha1"]


@pytest.mark.parametrize("misalign", [1, 2, 3])
@pytest.mark.parametrize("rec_len", [1500, 1501, 64, 77])
def test_unaligned_records(brb, orc, torch_dev, misalign, rec_len):
    n = 257
    data = workload.gen_records(0x5EED0003, 0, n, rec_len)
    d = torch_dev.zeros(data.size + 16, dtype=torch_dev.uint8, device="cuda")
    d[misalign:misalign + data.size] = to_dev(torch_dev, data)
    view = d[misalign:misalign + data.size]
    assert np.array_equal(brb.md5_batch_fixed(view, rec_len, n).cpu().numpy(), orc.md5_batch_fixed(data, rec_len, n))
    assert np.array_equal(brb.sha1_batch_fixed(view, rec_len, n).cpu().numpy(), orc.sha1_batch_fixed(data, rec_len, n))


def test_unaligned_output(brb, orc, torch_dev):
    n, L = 100, 1500
    data = to_dev(torch_dev, workload.gen_records(0x5EED0002, 0, n, L))
    out = torch_dev.zeros(n * 20 + 3, dtype=torch_dev.uint8, device="cuda")
    o5 = out[1:1 + 16 * n].view(n, 16)
    brb.md5_batch_fixed(data, L, n, out=o5)
    assert np.array_equal(o5.cpu().numpy(), orc.md5_batch_fixed(data.cpu().numpy(), L, n))
    o1 = out[3:3 + 20 * n].view(n, 20)
    brb.sha1_batch_fixed(data, L, n, out=o1)
    assert np.array_equal(o1.cpu().numpy(), orc.sha1_batch_fixed(data.cpu().numpy(), L, n))


def test_variable_records(brb, orc, torch_dev):
    rng = np.random.default_rng(11)
    n = 3000
    buf = workload.gen_records(0x5EED0005, 0, 1, 1 << 20)
    lens = rng.integers(0, 4000, n).astype(np.uint32)
    lens[:50] = 0
    lens[50:100] = rng.choice([55, 56, 63, 64, 65, 119, 120], 50)
    offs = rng.integers(0, buf.size - 4000, n).astype(np.uint64)      # overlapping, any alignment
    want5, want1 = orc.md5_batch(buf, offs, lens), orc.sha1_batch(buf, offs, lens)
    # host mode
    assert np.array_equal(brb.md5_batch(buf, offs, lens), want5)
    assert np.array_equal(brb.sha1_batch(buf, offs, lens), want1)
    # device mode
    d, o, ln = to_dev(torch_dev, buf), to_dev(torch_dev, offs.view(np.int64)), to_dev(torch_dev, lens.view(np.int32))
    assert np.array_equal(brb.md5_batch(d, o, ln).cpu().numpy(), want5)
    assert np.array_equal(brb.sha1_batch(d, o, ln).cpu().numpy(), want1)


def test_cfg2_full(brb, orc, torch_dev, golden):
    cfg = workload.CONFIGS[2]
    n, L = cfg["records"], cfg["rec_len"]
    data = workload.gen_records(workload.SEEDS[2], 0, n, L)
    d = to_dev(torch_dev, data)
    got5 = brb.md5_batch_fixed(d, L, n).cpu().numpy()
    got1 = brb.sha1_batch_fixed(d, L, n).cpu().numpy()
    assert np.array_equal(got5, orc.md5_batch_fixed(data, L, n, threads=16))
    assert np.array_equal(got1, orc.sha1_batch_fixed(data, L, n, threads=16))
    for e in golden["digests"]["configs"]["2"]["digests"]:
        assert got5[e["r"]].tobytes().hex() == e["md5"]
        assert got1[e["r"]].tobytes().hex() == e["sha1"]


def test_cfg3_full(brb, orc, torch_dev, golden):
    cfg = workload.CONFIGS[3]
    n, L = cfg["records"], cfg["rec_len"]
    data = workload.gen_records(workload.SEEDS[3], 0, n, L)
    got5 = brb.md5_batch_fixed(to_dev(torch_dev, data), L, n).cpu().numpy()
    assert np.array_equal(got5, orc.md5_batch_fixed(data, L, n, threads=16))
    for e in golden["digests"]["configs"]["3"]["digests"]:
        assert got5[e["r"]].tobytes().hex() == e["md5"]


@pytest.mark.parametrize("n,rec_len,off", [
    (65600, 1500, 0),        # line-aligned staging (digest_line.h), groups handed out by tickets
    (65600, 1500, 4),        # record bases 4 mod 16: every per-lane window shift changes
    (65601, 1532, 8),        # t = 60: two padding blocks; partial last group (per-DMA issue)
    (66000, 1508, 12),       # t = 36
    (65700, 132, 4),         # 3 lines per record, K = 2; < 160 B: per-DMA issue on every group
    (65600, 1504, 0),        # even dword stride
    (5000, 160, 4),          # smallest length with four DMAs per M0 write (instruction offsets)
    (5000, 156, 8),          # largest length without
    (3000, 1501, 0),         # not 4-byte multiple: record-relative stages (digest_dma.h), tickets
])
def test_large_batch_staging(brb, orc, torch_dev, n, rec_len, off):
    data = workload.gen_records(0x5EED0006, 0, n, rec_len)
    d = torch_dev.zeros(data.size + 64, dtype=torch_dev.uint8, device="cuda")
    d[off:off + data.size] = to_dev(torch_dev, data)
    view = d[off:off + data.size]
    assert np.array_equal(brb.md5_batch_fixed(view, rec_len, n).cpu().numpy(),
                          orc.md5_batch_fixed(data, rec_len, n, threads=16))
    assert np.array_equal(brb.sha1_batch_fixed(view, rec_len, n).cpu().numpy(),
                          orc.sha1_batch_fixed(data, rec_len, n, threads=16))


@pytest.mark.parametrize("kernel", [0, 1, 2, 3])
@pytest.mark.parametrize("n,off", [(1, 0), (64, 4), (65, 8), (4096 * 64 + 7, 0), (1 << 20, 12), (2048 * 4 * 64 * 3 + 65, 4)])
def test_b64_kernels_exact_buffer(brb, orc, torch_dev, kernel, n, off):
    """64-byte records (cfg3's shape) on each kernel the test option b64_kernel selects: 0 the
    generic DMA kernel, 1 the lean two-slot kernel, 2 / 3 the register-buffered one-slot kernel at 8
    / 4 waves per SIMD; partial last groups, several groups per wave, a buffer that ends at the batch."""
    data = workload.gen_records(0x5EED0010, 0, n, 64)
    d = torch_dev.zeros(off + data.size, dtype=torch_dev.uint8, device="cuda")
    d[off:] = to_dev(torch_dev, data)
    view = d[off:]
    with brb.TestOption("b64_kernel", kernel):
        got5 = brb.md5_batch_fixed(view, 64, n).cpu().numpy()
        got1 = brb.sha1_batch_fixed(view, 64, n).cpu().numpy()
    assert np.array_equal(got5, orc.md5_batch_fixed(data, 64, n, threads=16))
    assert np.array_equal(got1, orc.sha1_batch_fixed(data, 64, n, threads=16))


@pytest.mark.parametrize("n,rec_len,off", [
    (1, 4, 0), (63, 8, 4), (64, 64, 8), (65, 60, 12), (1000, 56, 0), (1001, 52, 4),
    (4097, 12, 0), (300_001, 32, 4), (270_000, 64, 0), (5000, 16, 8), (5000, 20, 0), (5000, 44, 12),
])
def test_short_records_exact_buffer(brb, orc, torch_dev, n, rec_len, off):
    """Records of at most 64 B at 4-byte bases (one compression + padding, or two when the tail
    holds 56..63 bytes) in a device buffer that ends exactly at the batch, so the staging's range
    check is what zeroes the bytes past the last record; n > 262 144 gives several groups per wave."""
    data = workload.gen_records(0x5EED000C, 0, n, rec_len)
    d = torch_dev.zeros(off + data.size, dtype=torch_dev.uint8, device="cuda")
    d[off:] = to_dev(torch_dev, data)
    view = d[off:]
    assert np.array_equal(brb.md5_batch_fixed(view, rec_len, n).cpu().numpy(),
                          orc.md5_batch_fixed(data, rec_len, n, threads=16))
    assert np.array_equal(brb.sha1_batch_fixed(view, rec_len, n).cpu().numpy(),
                          orc.sha1_batch_fixed(data, rec_len, n, threads=16))


def test_cfg5_full_shard(brb, orc, torch_dev, golden):
    """cfg5 as configured: GPU 7's whole shard of the 8 388 608-record batch (records [7/8 N, N),
    1 048 576 x 1500 B = 1.57 GB, HBM-resident), every digest against the oracle, and both ends of
    the shard against the hashlib golden digests (tests/golden/digests.json configs["5"])."""
    n_all, L = workload.CONFIGS[5]["records"], workload.CONFIGS[5]["rec_len"]
    r0, r1 = workload.shard(n_all, 7, 8)
    n = r1 - r0
    assert n == 1 << 20
    data = workload.gen_records(workload.SEEDS[5], r0, n, L)
    got = brb.md5_batch_fixed(to_dev(torch_dev, data), L, n).cpu().numpy()
    torch_dev.cuda.empty_cache()
    assert np.array_equal(got, orc.md5_batch_fixed(data, L, n, threads=16))
    seen = 0
    for e in golden["digests"]["configs"]["5"]["digests"]:
        if r0 <= e["r"] < r1:
            assert got[e["r"] - r0].tobytes().hex() == e["md5"]
            seen += 1
    assert seen == 66                # the last 64 records of cfg5 (which end the shard) + its first two


def test_cfg5_host_all_devices(brb, orc, golden):
    """cfg5's split as a C caller would run it on one node: one host-mode call with
    BRB_BATCH_ALL_DEVICES (contiguous ranges over every visible device; on a one-GPU box the split
    degenerates to that device).  A 262 144-record slice of GPU 0's shard, every digest vs the oracle."""
    n_all, L = workload.CONFIGS[5]["records"], workload.CONFIGS[5]["rec_len"]
    n = 1 << 18
    data = workload.gen_records(workload.SEEDS[5], 0, n, L)
    got = brb.md5_batch_fixed(data, L, n, all_devices=True)
    assert np.array_equal(got, orc.md5_batch_fixed(data, L, n, threads=16))
    for e in golden["digests"]["configs"]["5"]["digests"][:64]:
        assert got[e["r"]].tobytes().hex() == e["md5"]


@pytest.mark.parametrize("n,rec_len,off", [
    (65536, 1500, 0),        # cfg2's shape: one group per wave
    (5000, 68, 4),           # K = 1: the window of the prologue is the last one
    (5000, 128, 0),          # K = 1, t = 0: padding block only
    (5000, 192, 4),          # K = 2, nfull odd, t = 0: the last window's second half unused
    (300_001, 260, 8),       # several groups per wave, K = 3
])
def test_line_kernel_short_groups(brb, orc, torch_dev, n, rec_len, off):
    """The line-aligned kernel at K = 1 and 2 (two or three lines per record) and with several
    groups per wave, every digest against the oracle."""
    data = workload.gen_records(0x5EED0013, 0, n, rec_len)
    d = torch_dev.zeros(data.size + 64, dtype=torch_dev.uint8, device="cuda")
    d[off:off + data.size] = to_dev(torch_dev, data)
    view = d[off:off + data.size]
    assert np.array_equal(brb.md5_batch_fixed(view, rec_len, n).cpu().numpy(),
                          orc.md5_batch_fixed(data, rec_len, n, threads=16))
    assert np.array_equal(brb.sha1_batch_fixed(view, rec_len, n).cpu().numpy(),
                          orc.sha1_batch_fixed(data, rec_len, n, threads=16))


@pytest.mark.parametrize("rec_len,off", [
    (68, 4), (128, 8), (132, 12), (192, 0), (196, 4), (256, 8), (260, 12), (320, 0),
    (1024, 4), (1476, 8), (1500, 12), (1532, 0), (1540, 4),
])
def test_line_kernel_parities(brb, orc, torch_dev, rec_len, off):
    """The line kernel's launch-uniform choices (digest_line.h, round 6): K odd and even (slot P of a
    group's line 0), the tail in the last iteration's first or second block (TAIL_HI), no tail
    (t = 0), with the per-wave window and DMA tables shared by every group -- several groups per
    wave, a partial last group (300 001 records), buffer offsets 0/4/8/12, MD5 and SHA-1 against
    the oracle, two launches back to back."""
    n = 300_001
    data = workload.gen_records(0x5EED0015 ^ rec_len, 0, n, rec_len)
    d = torch_dev.zeros(data.size + 64, dtype=torch_dev.uint8, device="cuda")
    d[off:off + data.size] = to_dev(torch_dev, data)
    view = d[off:off + data.size]
    want = orc.md5_batch_fixed(data, rec_len, n, threads=16)
    for _ in range(2):
        assert np.array_equal(brb.md5_batch_fixed(view, rec_len, n).cpu().numpy(), want)
    assert np.array_equal(brb.sha1_batch_fixed(view, rec_len, n).cpu().numpy(),
                          orc.sha1_batch_fixed(data, rec_len, n, threads=16))


@pytest.mark.parametrize("rec_len", [1500, 1501])
def test_many_groups_per_wave(brb, orc, torch_dev, rec_len):
    """Batches large enough that every wave takes several 64-record groups from its workgroup's
    ticket counter (300 000 records = 4 688 groups over 2 048 wave slots): the line-staged kernel
    (1500 B) and the record-relative one (1501 B), every digest against the oracle."""
    n = 300_000
    data = workload.gen_records(0x5EED0005, 0, n, rec_len)
    d = to_dev(torch_dev, data)
    assert np.array_equal(brb.md5_batch_fixed(d, rec_len, n).cpu().numpy(),
                          orc.md5_batch_fixed(data, rec_len, n, threads=16))
    assert np.array_equal(brb.sha1_batch_fixed(d, rec_len, n).cpu().numpy(),
                          orc.sha1_batch_fixed(data, rec_len, n, threads=16))


# ---- Blowfish --------------------------------------------------------------------------------
@pytest.mark.parametrize("key", [b"TESTKEY", b"brb_framework_k4", bytes(range(56)), b"\xff" * 3])
@pytest.mark.parametrize("n_blocks", [1, 255, 256, 257, 10007])
def test_blowfish_batch_vs_oracle(brb, orc, torch_dev, key, n_blocks):
    ctx = brb.blowfish_init(key)
    oc = orc.bf_init(key)
    w = workload.gen_words(0x5EED0004, 2 * n_blocks)
    want = orc.bf_ecb(oc, w.copy())
    # host mode
    h = w.copy()
    brb.blowfish_encrypt_batch(ctx, h)
    assert np.array_equal(h, want)
    brb.blowfish_decrypt_batch(ctx, h)
    assert np.array_equal(h, w)
    # device mode (ctx uploaded once)
    cd = torch_dev.frombuffer(bytearray(brb.blowfish_ctx_bytes(ctx)), dtype=torch_dev.uint8).cuda()
    d = to_dev(torch_dev, w.view(np.int64))
    brb.blowfish_encrypt_batch(cd, d)
    assert np.array_equal(d.cpu().numpy().view(np.uint64), want)
    brb.blowfish_decrypt_batch(cd, d)
    assert np.array_equal(d.cpu().numpy().view(np.uint64), w)


def test_blowfish_kat_low_halves(brb, golden):
    for v in golden["kat"]["blowfish_ecb"]:
        ctx = brb.blowfish_init(bytes.fromhex(v["key"]))
        p = bytes.fromhex(v["plain"])
        w = np.array([int.from_bytes(p[:4], "big"), int.from_bytes(p[4:], "big")], np.uint64)
        brb.blowfish_encrypt_batch(ctx, w)
        got = (int(w[0]) & 0xFFFFFFFF).to_bytes(4, "big") + (int(w[1]) & 0xFFFFFFFF).to_bytes(4, "big")
        assert got.hex().upper() == v["cipher"]


def test_blowfish_golden_cfg4_prefix(brb, torch_dev, golden):
    g = golden["blowfish64"]["cfg4"]
    ctx = brb.blowfish_init(bytes.fromhex(g["key"]))
    w = workload.gen_words(g["seed"], 2 * g["pairs"])
    d = to_dev(torch_dev, w.view(np.int64))
    brb.blowfish_encrypt_batch(ctx, d)
    assert hashlib.sha256(d.cpu().numpy().tobytes()).hexdigest() == g["cipher_sha256"]


def test_cfg4_full_round_trip(brb, orc, torch_dev):
    """cfg4 at full size (65 536 x 16 KiB = 1 GiB): every ciphertext word == the 16-thread oracle
    (all 64 bits, the reference's carries included), and the exact 64-bit round trip restores every
    word."""
    cfg = workload.CONFIGS[4]
    n_words = cfg["records"] * cfg["rec_len"] // 8
    torch = torch_dev
    ctx = brb.blowfish_init(workload.CFG4_KEY)
    oc = orc.bf_init(workload.CFG4_KEY)
    w = workload.gen_words(workload.SEEDS[4], n_words)
    d = to_dev(torch, w.view(np.int64))
    cd = torch.frombuffer(bytearray(brb.blowfish_ctx_bytes(ctx)), dtype=torch.uint8).cuda()
    brb.blowfish_encrypt_batch(cd, d)
    want = orc.bf_ecb(oc, w.copy(), threads=16)
    assert np.array_equal(d.cpu().numpy().view(np.uint64), want)
    del want
    brb.blowfish_decrypt_batch(cd, d)
    assert torch.equal(d, to_dev(torch, w.view(np.int64)))


def test_beyond_4gib(brb, orc, torch_dev):
    """64-bit addressing end to end: one device buffer of 4.5 GiB, digested as 1500-byte records
    (3.2 M records, one call) and encrypted + decrypted as Blowfish blocks (302 M blocks, one call
    each way).  The records and blocks around byte offsets 2^31 and 2^32, the first and last ones
    and a random sample are checked against the oracle on host copies of just those slices; the
    round trip restores them."""
    torch = torch_dev
    total = 9 << 29
    words = torch.empty(total // 8, dtype=torch.int64, device="cuda")
    g = torch.Generator(device="cuda")
    g.manual_seed(0x4B1B)
    words.random_(generator=g)
    d = words.view(torch.uint8)
    L = 1500
    n = total // L
    rng = np.random.default_rng(3)
    recs = sorted(set(list(range(0, 64)) + list(range(n - 64, n)) + [int(x) for x in rng.integers(0, n, 200)]
                      + [o // L + k for o in (1 << 31, 1 << 32) for k in range(-3, 4)]))
    host = {r: d[r * L:(r + 1) * L].cpu().numpy() for r in recs}
    got5 = brb.md5_batch_fixed(d, L, n).cpu().numpy()
    got1 = brb.sha1_batch_fixed(d, L, n).cpu().numpy()
    for r in recs:
        assert got5[r].tobytes() == hashlib.md5(host[r].tobytes()).digest(), f"md5 record {r}"
        assert got1[r].tobytes() == hashlib.sha1(host[r].tobytes()).digest(), f"sha1 record {r}"
    del got5, got1
    # Blowfish over the same bytes: 16-byte blocks (two 64-bit words)
    nb = total // 16
    blocks = sorted(set(list(range(0, 16)) + list(range(nb - 16, nb)) + [int(x) for x in rng.integers(0, nb, 200)]
                        + [o // 16 + k for o in (1 << 31, 1 << 32) for k in range(-3, 4)]))
    plain = {b: words[2 * b:2 * b + 2].cpu().numpy().view(np.uint64).copy() for b in blocks}
    ctx = brb.blowfish_init(workload.CFG4_KEY)
    oc = orc.bf_init(workload.CFG4_KEY)
    cd = torch.frombuffer(bytearray(brb.blowfish_ctx_bytes(ctx)), dtype=torch.uint8).cuda()
    brb.blowfish_encrypt_batch(cd, words)
    for b in blocks:
        want = orc.bf_ecb(oc, plain[b].copy())
        assert np.array_equal(words[2 * b:2 * b + 2].cpu().numpy().view(np.uint64), want), f"block {b}"
    brb.blowfish_decrypt_batch(cd, words)
    for b in blocks:
        assert np.array_equal(words[2 * b:2 * b + 2].cpu().numpy().view(np.uint64), plain[b]), f"round trip {b}"
    del words, d
    torch.cuda.empty_cache()


def test_async_stream(brb, orc, torch_dev):
    torch = torch_dev
    n, L = 4096, 1500
    data = workload.gen_records(0x5EED0002, 0, n, L)
    s = torch.cuda.Stream()
    d = to_dev(torch, data)
    torch.cuda.synchronize()
    out = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
    brb.md5_batch_fixed(d, L, n, out=out, stream=s, async_=True)
    s.synchronize()
    assert np.array_equal(out.cpu().numpy(), orc.md5_batch_fixed(data, L, n))


def test_c_caller_batch_on_gpu(brb, tmp_path):
    from test_abi import build_caller, run_caller
    res = run_caller(build_caller(tmp_path))
    assert res["batch_md5_rc"] == "1"
    assert res["batch_md5_eq"] == "1" and res["batch_sha1_eq"] == "1" and res["batch_bf_eq"] == "1"
    assert res["batch_rc4_eq"] == "1"
    assert int(res["devices"]) >= 1 and res["per_device_md5_eq"] == "1"
    assert res["all_devices_md5_eq"] == "1" and res["all_devices_bf_eq"] == "1"
    assert res["set_device_out_of_range"] == "-1" and res["all_devices_with_device_ptrs"] == "-1"
    assert res["after_cleanup_md5_eq"] == "1"


def test_concurrent_host_threads(brb, orc, torch_dev):
    """§8(b) threading: the batch API is called from several event-loop threads at once (ctypes
    drops the GIL for the call).  Each thread has its own host-mode workspace and error string; the
    digests of every thread's batches must stay bit-exact, and a bad call in one thread must not
    leak its error into another."""
    import threading
    results, errors = {}, []

    def worker(t):
        try:
            for it in range(6):
                L = [1500, 64, 77, 1501][(t + it) % 4]
                n = 300 + 37 * t + it
                data = workload.gen_records(0x7A00 + t, it * 1000, n, L)
                if t == 3 and it == 2:
                    assert brb.lib().BRB_MD5BatchFixed(None, 64, 3, None, 0, None) == -1
                md5 = brb.md5_batch_fixed(data, L, n)
                sha = brb.sha1_batch_fixed(data, L, n)
                results[(t, it)] = (np.array_equal(md5, orc.md5_batch_fixed(data, L, n)),
                                    np.array_equal(sha, orc.sha1_batch_fixed(data, L, n)))
                assert brb.lib().BRB_CryptoGPU_LastError() == b""
        except Exception as e:          # surfaced in the main thread below
            errors.append(repr(e))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=100)
    assert not errors, errors
    assert len(results) == 24 and all(a and b for a, b in results.values())


@pytest.mark.gpu
@pytest.mark.parametrize("n,max_len,seed", [(70_001, 3000, 1), (5_000, 200, 2), (3_000, 20_000, 3)])
def test_variable_records_line_kernel(brb, orc, torch_dev, n, max_len, seed):
    """BRB_MD5Batch / BrbSha1_Batch through the line-staged variable-length kernel
    (digest_var_line.h): every byte alignment, overlapping records, empty records, groups whose
    records differ in length by up to max_len; host, device and all-devices modes vs the oracle."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, max_len + 1, n).astype(np.uint32)
    lens[rng.integers(0, n, n // 20)] = 0
    span = int(lens.astype(np.uint64).sum() // 2 + max_len + 64)
    offs = rng.integers(0, span - max_len, n).astype(np.uint64)          # overlapping, any byte
    buf = workload.gen_records(0x5EED0011 + seed, 0, 1, span)
    want5, want1 = orc.md5_batch(buf, offs, lens), orc.sha1_batch(buf, offs, lens)
    assert np.array_equal(brb.md5_batch(buf, offs, lens), want5)
    assert np.array_equal(brb.sha1_batch(buf, offs, lens), want1)
    d, o, ln = to_dev(torch_dev, buf), to_dev(torch_dev, offs.view(np.int64)), to_dev(torch_dev, lens.view(np.int32))
    assert np.array_equal(brb.md5_batch(d, o, ln).cpu().numpy(), want5)
    assert np.array_equal(brb.sha1_batch(d, o, ln).cpu().numpy(), want1)
    assert np.array_equal(brb.md5_batch(buf, offs, lens, all_devices=True), want5)


def _lens_shape(kind, n, rng):
    if kind == "equal":
        return np.full(n, 1500, np.uint32)
    if kind == "bimodal":
        return rng.choice(np.array([0, 4000], np.uint32), n)
    if kind == "wide":
        return (rng.random(n) ** 3 * 100_000).astype(np.uint32)           # long tail: scaled buckets
    if kind == "descending":
        return np.linspace(3000, 0, n).astype(np.uint32)
    return rng.integers(1000, 2001, n).astype(np.uint32)                   # the md5var bench shape


@pytest.mark.gpu
@pytest.mark.parametrize("sort", [1, 0, 2])
@pytest.mark.parametrize("n,kind", [(1, "uniform"), (64, "uniform"), (65, "bimodal"), (255, "wide"), (256, "uniform"),
                                    (257, "descending"), (1000, "equal"), (4097, "bimodal"), (9001, "wide"),
                                    (65536, "uniform"), (140_001, "bimodal"), (300_000, "uniform")])
def test_variable_records_bucketed(brb, orc, torch_dev, n, kind, sort):
    """Length bucketing of BRB_MD5Batch / BrbSha1_Batch (digest_var_line.h sorted_record): inside
    every chunk of 256 records the groups are formed by length bucket, and each digest must still
    land in its record's slot.  Bucketing applies past the first round of tickets (more than
    2 048 groups on 256 CUs), so the two largest shapes exercise it; the others check the caller-order
    path the same way.  Chunk edges (n not a multiple of 64 or 256, a last chunk with fewer
    groups), equal lengths, two far-apart lengths, a long tail (scaled buckets), descending lengths
    and the bench's U[1000, 2000]; "var_sort" on and off (caller-order groups) vs the oracle."""
    rng = np.random.default_rng(n * 7 + len(kind))
    lens = _lens_shape(kind, n, rng)
    span = int(lens.astype(np.uint64).sum() + 64 * n + 4096)
    offs = np.cumsum(rng.integers(0, 64, n).astype(np.uint64) + np.concatenate([[0], lens[:-1]]).astype(np.uint64))
    offs = offs.astype(np.uint64)
    buf = workload.gen_records(0x5EED0014, n, 1, span)
    want5 = orc.md5_batch(buf, offs, lens, threads=16)
    want1 = orc.sha1_batch(buf, offs, lens, threads=16)
    d, o, ln = to_dev(torch_dev, buf), to_dev(torch_dev, offs.view(np.int64)), to_dev(torch_dev, lens.view(np.int32))
    with brb.TestOption("var_sort", sort):
        assert np.array_equal(brb.md5_batch(d, o, ln).cpu().numpy(), want5)
        assert np.array_equal(brb.sha1_batch(d, o, ln).cpu().numpy(), want1)
        assert np.array_equal(brb.md5_batch(buf, offs, lens), want5)


@pytest.mark.gpu
@pytest.mark.parametrize("sort", [1, 2])
@pytest.mark.parametrize("pc,short", [(1, 0), (2, 5), (3, 0), (3, 63)])
def test_variable_records_bucketed_partial_chunk(brb, orc, torch_dev, pc, short, sort):
    """the last chunk of a bucketed batch holds pc < 4 groups and its round
    t = g / CUs is not a multiple of 4.  The slice rotation must stay inside the pc slices that
    hold records (the round-3 kernel rotated over all 4, so a group took an empty slice and 64
    records were never digested).  n = 64 (9 CUs + pc) - short puts the last chunk at round 9 on
    any CU count; every digest is checked against the oracle, with var_sort 1 and 2."""
    cus = torch_dev.cuda.get_device_properties(0).multi_processor_count
    n = 64 * (9 * cus + pc) - short
    rng = np.random.default_rng(1000 * pc + short)
    lens = rng.integers(100, 700, n).astype(np.uint32)
    offs = (np.cumsum(lens.astype(np.uint64)) - lens).astype(np.uint64)
    buf = workload.gen_records(0x5EED0015, n, 1, int(lens.astype(np.uint64).sum()) + 64)
    want = orc.md5_batch(buf, offs, lens, threads=16)
    d, o, ln = to_dev(torch_dev, buf), to_dev(torch_dev, offs.view(np.int64)), to_dev(torch_dev, lens.view(np.int32))
    with brb.TestOption("var_sort", sort):
        got = brb.md5_batch(d, o, ln).cpu().numpy()
        bad = np.nonzero(~np.all(got == want, axis=1))[0]
        assert bad.size == 0, f"{bad.size} digests differ, first at record {bad[:4]} of {n}"
        assert np.array_equal(brb.sha1_batch(d, o, ln).cpu().numpy(), orc.sha1_batch(buf, offs, lens, threads=16))


@pytest.mark.gpu
def test_variable_records_wide_span(brb, orc, torch_dev):
    """Groups whose records lie more than 2 GiB apart (32-bit DMA offsets cannot reach them) are
    digested by the per-lane path inside the same launch; the other groups stay line-staged."""
    far = (1 << 31) + 12345
    n = 640
    rng = np.random.default_rng(12)
    lens = rng.integers(0, 3000, n).astype(np.uint32)
    offs = rng.integers(0, 1 << 20, n).astype(np.uint64)
    offs[::7] += far                                                     # every group spans > 2 GiB
    offs[128:192] = rng.integers(0, 1 << 20, 64).astype(np.uint64)       # one group does not
    d = torch_dev.empty(far + (1 << 20) + 4096, dtype=torch_dev.uint8, device="cuda")
    lo_h = workload.gen_records(0x5EED0012, 0, 1, (1 << 20) + 4096)
    hi_h = workload.gen_records(0x5EED0013, 0, 1, (1 << 20) + 4096)
    d[: lo_h.size] = to_dev(torch_dev, lo_h)
    d[far: far + hi_h.size] = to_dev(torch_dev, hi_h)
    got5 = brb.md5_batch(d, to_dev(torch_dev, offs.view(np.int64)), to_dev(torch_dev, lens.view(np.int32))).cpu().numpy()
    for i in range(n):
        o, L = int(offs[i]), int(lens[i])
        src = hi_h[o - far: o - far + L] if o >= far else lo_h[o: o + L]
        assert got5[i].tobytes() == hashlib.md5(src.tobytes()).digest(), i
    del d
