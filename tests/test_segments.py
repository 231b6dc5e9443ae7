"""MD5 of segment lists: the MetaData pack digest (meta_data.c:397-433: Init,
UpdateBig per item, Final) batched as BRB_MD5BatchSegments, against the oracle's streaming MD5 (and
hashlib) on the concatenation of each record's segments."""
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


def _case(seed, n_rec, max_segs, max_len):
    rng = np.random.default_rng(seed)
    seg_counts = rng.integers(0, max_segs + 1, n_rec)
    first = np.zeros(n_rec + 1, np.uint64)
    first[1:] = np.cumsum(seg_counts)
    nseg = int(first[-1])
    lens = rng.integers(0, max_len + 1, nseg).astype(np.uint32)
    lens[rng.random(nseg) < 0.2] = rng.integers(0, 4, int((rng.random(nseg) < 0.2).sum()) or 1)[0]
    pool = workload.gen_records(0x5EED00F4 + seed, 0, 1, int(lens.sum()) + 4096)
    offs = rng.integers(0, pool.size - max_len - 1, nseg).astype(np.uint64)   # scattered, overlapping
    return pool, offs, lens, first


def _want(orc, pool, offs, lens, first):
    out = []
    for i in range(len(first) - 1):
        msg = b"".join(pool[int(offs[k]):int(offs[k]) + int(lens[k])].tobytes()
                       for k in range(int(first[i]), int(first[i + 1])))
        out.append(hashlib.md5(msg).digest())
    return np.frombuffer(b"".join(out), np.uint8).reshape(-1, 16)


@pytest.mark.parametrize("seg_line,slots", [(1, 2), (1, 3), (2, 0), (0, 0)])
@pytest.mark.parametrize("seed,n_rec,max_segs,max_len", [(1, 300, 5, 40), (2, 200, 20, 7), (3, 64, 3, 3000),
                                                        (4, 1000, 1, 200), (5, 5, 200, 100), (6, 700, 40, 3),
                                                        (7, 257, 8, 130)])
def test_segments_vs_hashlib(brb, orc, torch_dev, seed, n_rec, max_segs, max_len, seg_line, slots):
    """seg_line 1: the line-staged kernel (line_stream.h; round 4) with a ring of `slots` LDS-DMA
    slots (test option line_slots), 2: its producer / consumer wave-pair form, 0: the per-lane block
    kernel."""
    pool, offs, lens, first = _case(seed, n_rec, max_segs, max_len)
    want = _want(orc, pool, offs, lens, first)
    with brb.TestOption("seg_line", seg_line), brb.TestOption("line_slots", slots):
        got = brb.md5_batch_segments(pool, offs, lens, first)
        assert np.array_equal(got, want)
        t = torch_dev
        dev = brb.md5_batch_segments(t.from_numpy(pool).cuda(), t.from_numpy(offs).cuda(), t.from_numpy(lens).cuda(),
                                     t.from_numpy(first).cuda())
        assert np.array_equal(dev.cpu().numpy(), want)


def _pack_items_case(n, K, Q, gap, seed):
    """The md5seg bench layout: record i = K items of Q bytes inside one pack, `gap` bytes between
    items (the 24-byte item fields and the canary: 25), packs back to back."""
    rng = np.random.default_rng(seed)
    stride = 64 + K * (gap + Q)
    pool = workload.gen_records(0x5EED00F6 + seed, 0, 1, n * stride + 64)
    offs = (np.arange(n, dtype=np.uint64)[:, None] * stride + 64 + gap - 1
            + np.arange(K, dtype=np.uint64)[None, :] * (gap + Q)).reshape(-1).astype(np.uint64)
    lens = np.full(n * K, Q, np.uint32)
    if seed % 2:                                  # ragged item sizes inside the same slots
        lens = rng.integers(0, Q + 1, n * K).astype(np.uint32)
    first = (np.arange(n + 1, dtype=np.uint64) * K).astype(np.uint64)
    return pool, offs, lens, first


@pytest.mark.parametrize("n,K,Q,gap,seed", [(65536, 4, 375, 25, 0), (4097, 4, 375, 25, 1), (3000, 9, 61, 3, 2),
                                            (2000, 3, 700, 130, 3), (1024, 16, 4, 1, 4), (640, 2, 1, 0, 5)])
@pytest.mark.parametrize("seg_line", [1, 2])
def test_segments_pack_layout(brb, orc, torch_dev, n, K, Q, gap, seed, seg_line):
    """Segments as the MetaData items of back-to-back packs (the md5seg bench shape at full size
    and variants: ragged sizes, items sharing memory lines, 1..4-byte items), line-staged kernel vs
    the per-lane kernel vs hashlib on sampled records (every record for the smaller shapes)."""
    t = torch_dev
    pool, offs, lens, first = _pack_items_case(n, K, Q, gap, seed)
    dev = lambda a: t.from_numpy(np.ascontiguousarray(a)).cuda()   # noqa: E731
    d, o, ln, fi = dev(pool), dev(offs), dev(lens), dev(first)
    with brb.TestOption("seg_line", seg_line):
        got = brb.md5_batch_segments(d, o, ln, fi).cpu().numpy()
    with brb.TestOption("seg_line", 0):
        ref = brb.md5_batch_segments(d, o, ln, fi).cpu().numpy()
    assert np.array_equal(got, ref)
    idx = range(n) if n <= 4097 else list(range(0, n, 97)) + [n - 1]
    for i in idx:
        msg = b"".join(pool[int(offs[k]):int(offs[k]) + int(lens[k])].tobytes()
                       for k in range(int(first[i]), int(first[i + 1])))
        assert got[i].tobytes() == hashlib.md5(msg).digest(), i


@pytest.mark.parametrize("seg_line", [1, 2])
def test_segments_mixed_wide_groups(brb, torch_dev, seg_line):
    """One launch with groups whose segments lie within 2 GiB (line-staged) and groups whose
    segments lie more than 2 GiB apart (32-bit DMA offsets cannot reach: the per-lane path), 640
    records in 10 groups, every other group wide."""
    t = torch_dev
    far = (1 << 31) + 4099
    size = far + (1 << 20)
    d = t.empty(size, dtype=t.uint8, device="cuda")
    lo_h = workload.gen_records(0x5EED00F7, 0, 1, 1 << 20)
    hi_h = workload.gen_records(0x5EED00F8, 0, 1, 1 << 20)
    d[: lo_h.size] = t.from_numpy(lo_h).cuda()
    d[far:far + hi_h.size] = t.from_numpy(hi_h).cuda()
    rng = np.random.default_rng(41)
    n = 640
    counts = rng.integers(1, 5, n)
    first = np.zeros(n + 1, np.uint64)
    first[1:] = np.cumsum(counts)
    nseg = int(first[-1])
    lens = rng.integers(0, 900, nseg).astype(np.uint32)
    offs = rng.integers(0, (1 << 20) - 1000, nseg).astype(np.uint64)
    wide = np.zeros(nseg, bool)
    for g in range(1, 10, 2):                    # groups 1, 3, 5, 7, 9: one segment far away
        r = 64 * g + 5
        wide[int(first[r])] = True
    offs[wide] += far
    dev = lambda a: t.from_numpy(np.ascontiguousarray(a)).cuda()   # noqa: E731
    with brb.TestOption("seg_line", seg_line):
        got = brb.md5_batch_segments(d, dev(offs), dev(lens), dev(first)).cpu().numpy()
    for i in range(n):
        parts = []
        for k in range(int(first[i]), int(first[i + 1])):
            o, m = int(offs[k]), int(lens[k])
            parts.append((hi_h[o - far:o - far + m] if o >= far else lo_h[o:o + m]).tobytes())
        assert got[i].tobytes() == hashlib.md5(b"".join(parts)).digest(), i
    del d
    t.cuda.empty_cache()


@pytest.mark.parametrize("seg_line", [1, 2])
def test_segments_many_groups_per_wave(brb, torch_dev, seg_line):
    """More groups than the launch has waves (line kernel) or wave pairs (pair kernel): 200 000
    records = 3 125 groups on at most 1 024, so each wave / pair runs three or four groups in
    sequence and the pair protocol's events carry over from group to group.  Every seventh group is
    wide (one segment past 2 GiB: the per-lane path, in the pair kernel the producer alone), so one
    pair's sequence mixes planned groups and groups it runs alone.  Every record against the
    per-lane kernel, a sample (all wide groups among it) against hashlib."""
    t = torch_dev
    far = (1 << 31) + 4099
    size = far + (1 << 20)
    d = t.empty(size, dtype=t.uint8, device="cuda")
    lo_h = workload.gen_records(0x5EED00F9, 0, 1, 1 << 20)
    hi_h = workload.gen_records(0x5EED00FA, 0, 1, 1 << 20)
    d[: lo_h.size] = t.from_numpy(lo_h).cuda()
    d[far:far + hi_h.size] = t.from_numpy(hi_h).cuda()
    rng = np.random.default_rng(43)
    n = 200_000
    groups = (n + 63) // 64
    wide_rec = [64 * g + 11 for g in range(3, groups, 7)]
    counts = rng.integers(0, 4, n)
    counts[wide_rec] = np.maximum(counts[wide_rec], 1)
    first = np.zeros(n + 1, np.uint64)
    first[1:] = np.cumsum(counts)
    nseg = int(first[-1])
    lens = rng.integers(0, 400, nseg).astype(np.uint32)
    offs = rng.integers(0, (1 << 20) - 500, nseg).astype(np.uint64)
    offs[first[wide_rec].astype(np.int64)] += np.uint64(far)
    dev = lambda a: t.from_numpy(np.ascontiguousarray(a)).cuda()   # noqa: E731
    o, ln, fi = dev(offs), dev(lens), dev(first)
    with brb.TestOption("seg_line", seg_line):
        got = brb.md5_batch_segments(d, o, ln, fi).cpu().numpy()
    with brb.TestOption("seg_line", 0):
        ref = brb.md5_batch_segments(d, o, ln, fi).cpu().numpy()
    assert np.array_equal(got, ref)
    for i in sorted(set(wide_rec) | set(range(0, n, 211)) | {n - 1}):
        parts = []
        for k in range(int(first[i]), int(first[i + 1])):
            a, m = int(offs[k]), int(lens[k])
            parts.append((hi_h[a - far:a - far + m] if a >= far else lo_h[a:a + m]).tobytes())
        assert got[i].tobytes() == hashlib.md5(b"".join(parts)).digest(), i
    del d
    t.cuda.empty_cache()


@pytest.mark.gpu
@pytest.mark.parametrize("seg_line", [1, 2])
def test_segments_long_lane_in_wide_group(brb, torch_dev, seg_line):
    """A group whose lines span more than 2 GiB takes the per-lane path (in the wave-pair kernel: the
    producer alone, its partner waiting for the next plan); one of its lanes digests a 96 MiB segment
    -- far longer than a wait without progress may last -- so the waiting wave must see the
    producer's heartbeat.  128 records: group 0 wide with the long lane, group 1 ordinary."""
    t = torch_dev
    far = (1 << 31) + 4099
    big = 96 << 20
    size = (far + big + 4096 + 7) // 8 * 8
    d = t.empty(size, dtype=t.uint8, device="cuda")
    g = t.Generator(device="cuda")
    g.manual_seed(0x10C)
    d.view(t.int64).random_(generator=g)
    n = 128
    first = np.arange(n + 1, dtype=np.uint64) * 2
    offs = (np.arange(2 * n, dtype=np.uint64) * 1000).astype(np.uint64)
    lens = np.full(2 * n, 700, np.uint32)
    offs[1], lens[1] = far, big                 # record 0: one segment past 2 GiB, 96 MiB long
    offs[3] = far + 5                           # record 1 too: the group spans > 2 GiB
    dev = lambda a: t.from_numpy(np.ascontiguousarray(a)).cuda()   # noqa: E731
    with brb.TestOption("seg_line", seg_line):
        got = brb.md5_batch_segments(d, dev(offs), dev(lens), dev(first)).cpu().numpy()
    for i in list(range(0, 4)) + [64, 100, 127]:
        msg = b"".join(d[int(offs[k]):int(offs[k]) + int(lens[k])].cpu().numpy().tobytes()
                       for k in range(int(first[i]), int(first[i + 1])))
        assert got[i].tobytes() == hashlib.md5(msg).digest(), i
    del d
    t.cuda.empty_cache()


@pytest.mark.gpu
@pytest.mark.parametrize("seg_line", [1, 2])
def test_segments_long_empty_run_per_lane(brb, torch_dev, seg_line):
    """A record of 1.5 million empty segments and then one with bytes: its group holds more segments
    than the wave's table, so it takes the per-lane path (in the wave-pair kernel the producer alone,
    its partner waiting).  Skipping the empty run emits no block, and outlasts a wait without progress
    unless the walk beats per skipped segment.  128 records vs hashlib."""
    t = torch_dev
    rng = np.random.default_rng(53)
    pool = workload.gen_records(0x5EED00FC, 0, 1, 1 << 20)
    E, n = 1_500_000, 128
    counts = np.array([E + 1] + [2] * (n - 1), np.uint64)
    first = np.zeros(n + 1, np.uint64)
    first[1:] = np.cumsum(counts)
    nseg = int(first[-1])
    lens = np.zeros(nseg, np.uint32)
    offs = np.zeros(nseg, np.uint64)
    lens[E] = 100
    offs[E] = 4097
    lens[E + 1:] = rng.integers(1, 1200, nseg - E - 1).astype(np.uint32)
    offs[E + 1:] = rng.integers(0, (1 << 20) - 1200, nseg - E - 1).astype(np.uint64)
    dev = lambda a: t.from_numpy(np.ascontiguousarray(a)).cuda()   # noqa: E731
    with brb.TestOption("seg_line", seg_line):
        got = brb.md5_batch_segments(dev(pool), dev(offs), dev(lens), dev(first)).cpu().numpy()
    for i in range(n):
        msg = b"".join(pool[int(offs[k]):int(offs[k]) + int(lens[k])].tobytes()
                       for k in range(max(int(first[i]), E), int(first[i + 1])))
        assert got[i].tobytes() == hashlib.md5(msg).digest(), i


def test_segments_equal_streaming_oracle(brb, orc):
    """The oracle's BRB_MD5Init/UpdateBig/Final restatement over the items = the batch digest."""
    import ctypes
    pool, offs, lens, first = _case(9, 50, 6, 100)
    got = brb.md5_batch_segments(pool, offs, lens, first)
    for i in range(50):
        c = orc.Md5Ctx()
        orc.lib().orc_md5_init(ctypes.byref(c))
        for k in range(int(first[i]), int(first[i + 1])):
            seg = pool[int(offs[k]):int(offs[k]) + int(lens[k])].tobytes()
            orc.lib().orc_md5_update_big(ctypes.byref(c), seg, len(seg))
        orc.lib().orc_md5_final(ctypes.byref(c))
        assert bytes(c.digest) == got[i].tobytes()


def test_segments_empty_and_sub_ranges(brb):
    pool = np.arange(100, dtype=np.uint8)
    # records: no segments, one empty segment, one segment; first[] not starting at 0
    first = np.array([3, 3, 4, 5], np.uint64)
    offs = np.array([0, 0, 0, 50, 10], np.uint64)
    lens = np.array([9, 9, 9, 0, 33], np.uint32)
    got = brb.md5_batch_segments(pool, offs, lens, first)
    assert got[0].tobytes() == hashlib.md5(b"").digest()
    assert got[1].tobytes() == hashlib.md5(b"").digest()
    assert got[2].tobytes() == hashlib.md5(pool[10:43].tobytes()).digest()


@pytest.mark.parametrize("seg_line", [1, 2])
def test_segments_at_buffer_ends(brb, orc, torch_dev, seg_line):
    """Segments that start at the device buffer's first byte (a range that would begin up to 3
    bytes before it) and end at its last byte, in a buffer of exactly the pool's size; 130 records
    (a partial last wave), lengths 1..200."""
    rng = np.random.default_rng(17)
    n_rec = 130
    pool = workload.gen_records(0x5EED00F5, 0, 1, 20001)
    counts = rng.integers(1, 6, n_rec)
    first = np.zeros(n_rec + 1, np.uint64)
    first[1:] = np.cumsum(counts)
    nseg = int(first[-1])
    lens = rng.integers(1, 201, nseg).astype(np.uint32)
    offs = np.array([rng.integers(0, pool.size - int(n) + 1) for n in lens], np.uint64)
    ends = rng.random(nseg)
    offs[ends < 0.2] = 0
    sel = ends > 0.8
    offs[sel] = pool.size - lens[sel]
    want = _want(orc, pool, offs, lens, first)
    t = torch_dev
    with brb.TestOption("seg_line", seg_line):
        dev = brb.md5_batch_segments(t.from_numpy(pool).cuda(), t.from_numpy(offs).cuda(), t.from_numpy(lens).cuda(),
                                     t.from_numpy(first).cuda())
    assert np.array_equal(dev.cpu().numpy(), want)


@pytest.mark.parametrize("seg_line", [1, 2])
def test_segments_beyond_4gib(brb, torch_dev, seg_line):
    """Segment offsets past 2^32 in one 4.5 GiB device buffer: 500 records of 1..6 segments
    (0..700 bytes), some straddling byte offsets 2^31 and 2^32, against hashlib on host copies of
    just those segments."""
    t = torch_dev
    total = 9 << 29
    words = t.empty(total // 8, dtype=t.int64, device="cuda")
    g = t.Generator(device="cuda")
    g.manual_seed(0x4B1E)
    words.random_(generator=g)
    d = words.view(t.uint8)
    rng = np.random.default_rng(31)
    n_rec = 500
    counts = rng.integers(1, 7, n_rec)
    first = np.zeros(n_rec + 1, np.uint64)
    first[1:] = np.cumsum(counts)
    nseg = int(first[-1])
    lens = rng.integers(0, 701, nseg).astype(np.uint32)
    offs = rng.integers(0, total - 701, nseg).astype(np.uint64)
    for i, o in enumerate([(1 << 31) - 300, (1 << 32) - 300, (1 << 32) - 1, (1 << 32) + 2, total - 700]):
        offs[i], lens[i] = o, 700
    segs = [d[int(o):int(o) + int(m)].cpu().numpy().tobytes() for o, m in zip(offs, lens)]
    dev = lambda a: t.from_numpy(np.ascontiguousarray(a)).cuda()   # noqa: E731
    with brb.TestOption("seg_line", seg_line):
        got = brb.md5_batch_segments(d, dev(offs), dev(lens), dev(first)).cpu().numpy()
    for i in range(n_rec):
        msg = b"".join(segs[k] for k in range(int(first[i]), int(first[i + 1])))
        assert got[i].tobytes() == hashlib.md5(msg).digest(), i
    del words, d
    t.cuda.empty_cache()


@pytest.mark.parametrize("device", [False, True])
def test_segments_pair_fault_reported(brb, torch_dev, device):
    """A protocol fault in the producer / consumer pair (test option pair_stall: the first pair never
    posts its first plan, so the consumer's and then the producer's bounded waits give up) makes the
    call fail with BRB_BATCH_FAULT (-4, pair_fault.h) instead of returning digests; the next call on
    the same thread is clean and equals hashlib."""
    t = torch_dev
    n = 256
    pool = workload.gen_records(0x5EED00FB, 0, 1, 1 << 20)
    rng = np.random.default_rng(47)
    first = (np.arange(n + 1, dtype=np.uint64) * 2).astype(np.uint64)
    lens = rng.integers(600, 1200, 2 * n).astype(np.uint32)      # > 46 ring words per lane: the producer blocks
    offs = rng.integers(0, (1 << 20) - 1200, 2 * n).astype(np.uint64)
    args = (pool, offs, lens, first)
    if device:
        args = tuple(t.from_numpy(np.ascontiguousarray(a)).cuda() for a in args)
    with brb.TestOption("seg_line", 2), brb.TestOption("pair_stall", 1):
        with pytest.raises(RuntimeError, match=r"returned -4: wave-pair protocol fault"):
            brb.md5_batch_segments(*args)
    with brb.TestOption("seg_line", 2):
        got = brb.md5_batch_segments(*args)
    got = got.cpu().numpy() if device else got
    for i in range(n):
        msg = b"".join(pool[int(offs[k]):int(offs[k]) + int(lens[k])].tobytes() for k in (2 * i, 2 * i + 1))
        assert got[i].tobytes() == hashlib.md5(msg).digest(), i
