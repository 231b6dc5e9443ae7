"""MetaData packs: MetaDataPack / MetaDataUnpack (meta_data.c:104-328) in batches.

CPU: the oracle's pack layout and digest against struct + hashlib; the oracle's unpack against a
second, pure-Python restatement of meta_data.c:145-328 (py_unpack below) on a corpus of valid and
mutated packs that reaches every return code; the reference's quirks.  GPU: BRB_MetaDataUnpackBatch
(host, device and all-devices modes, packs at arbitrary byte offsets) against the oracle on every
field of every pack, and metadata.pack_batch against the oracle's pack byte for byte.

Parity: the digest is pinned by hashlib; the control flow and the unsigned-long arithmetic of the
MetaDataUnpackerInfo fields rest on the two restatements (no reference-run vector exists).
"""
import hashlib
import struct

import numpy as np
import pytest

M64 = 1 << 64


def py_unpack(pack: bytes):
    """meta_data.c:145-328 restated in Python (bytes past the pack read as 0; an item larger than
    the whole pack is not read -- include/brb_crypto.h).  -> (code, items, cur_offset, cur_remaining,
    cur_needed)."""
    size = len(pack)
    byte = lambda p: pack[p] if p < size else 0
    field = lambda p, n: bytes(byte(p + k) for k in range(n))
    if field(16, 8) != b"BRB_META":                                   # :183-195
        return (0, 0, 0, 0, 0)
    count = struct.unpack("<i", field(4, 4))[0]
    off, rem, need, n, h = 64, 0, 0, 0, hashlib.md5()                 # :198-199
    for _ in range(max(count, 0)):                                    # :202
        rem = (size - off) % M64                                      # :213
        if rem < 32:                                                  # :216-224 sizeof(MetaDataItem)
            return (5, n, off, rem, (32 - rem) % M64)
        sz = int.from_bytes(field(off + 16, 8), "little")
        off, rem = off + 24, (rem - 24) % M64                          # :227-232
        if rem < (sz + 1) % M64 or sz > size:                         # :237-246
            return (6, n, off, rem, (sz + 1 - rem) % M64)
        h.update(field(off, sz))                                      # :249-254
        off, rem = off + sz, (rem - sz) % M64
        if byte(off) != 0x1F:                                         # :258-268
            return (3, n, off, rem, need)
        off, rem, n = off + 1, (rem - 1) % M64, n + 1                   # :271-277
        if off == size:                                               # :280-281
            break
    return (7 if h.digest() == field(24, 16) else 4, n, off, rem, need)   # :285-298


def build(items) -> bytes:
    """MetaDataPack by struct (libbrb_data.h:313-330 LP64 layout), digest by hashlib."""
    body = b"".join(struct.pack("<QQQ", i, s, len(d)) + d + b"\x1f" for i, s, d in items)
    dig = hashlib.md5(b"".join(d for _, _, d in items)).digest()
    return struct.pack("<iiQ8s16s24s", 0, len(items), len(body), b"BRB_META", dig, bytes(24)) + body


def random_items(rng, max_items=6, max_len=200):
    k = int(rng.integers(0, max_items + 1))
    out = []
    for j in range(k):
        n = int(rng.integers(0, 7)) if (j == k - 1 and rng.random() < 0.3) else int(rng.integers(0, max_len))
        out.append((int(rng.integers(0, M64, dtype=np.uint64)), int(rng.integers(0, 1 << 20)),
                    rng.integers(0, 256, n, dtype=np.uint8).tobytes()))
    return out


def item_field_pos(items, j):
    """Byte position of item j's sz field."""
    return 64 + sum(24 + len(d) + 1 for _, _, d in items[:j]) + 16


def mutate(rng, items, pack: bytes) -> bytes:
    b = bytearray(pack)
    kind = int(rng.integers(0, 9))
    if kind == 0:                                                     # truncated anywhere
        return bytes(b[: int(rng.integers(0, len(b)))])
    if kind == 1 and items:                                           # a canary flipped
        j = int(rng.integers(0, len(items)))
        b[item_field_pos(items, j) + 8 + len(items[j][2])] ^= 0x40
    elif kind == 2 and any(d for _, _, d in items):                   # a data byte flipped
        j = next(j for j, (_, _, d) in enumerate(items) if d)
        b[item_field_pos(items, j) + 8] ^= 1
    elif kind == 3:                                                   # magic broken
        b[16 + int(rng.integers(0, 8))] ^= 0x20
    elif kind == 4:                                                   # item_count off
        b[4:8] = struct.pack("<i", int(rng.integers(-2, len(items) + 4)))
    elif kind == 5 and items:                                         # an sz field off
        j = int(rng.integers(0, len(items)))
        sz = len(items[j][2])
        v = [M64 - 1, int(rng.integers(0, M64, dtype=np.uint64)), sz + 1, max(sz - 1, 0), len(b) + 5,
             len(b)][int(rng.integers(0, 6))]
        p = item_field_pos(items, j)
        b[p:p + 8] = struct.pack("<Q", v % M64)
    elif kind == 6:                                                   # trailing bytes
        b += rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8).tobytes()
    elif kind == 7:                                                   # shorter than the header
        return bytes(b[: int(rng.integers(0, 64))])
    return bytes(b)


def corpus(seed, n):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        items = random_items(rng)
        p = build(items)
        out.append(p if rng.random() < 0.35 else mutate(rng, items, p))
    return out


# ---- CPU ----------------------------------------------------------------------------------------
def test_oracle_pack_layout_and_digest(orc):
    rng = np.random.default_rng(1)
    for _ in range(200):
        items = random_items(rng)
        assert orc.metadata_pack(items) == build(items)


def test_unpack_two_restatements_agree(orc):
    packs = corpus(2, 3000)
    codes = set()
    for p in packs:
        got = orc.metadata_unpack(p)
        assert got == py_unpack(p), p.hex()
        codes.add(got[0])
    assert codes == {0, 3, 4, 5, 6, 7}, codes           # every code the reference can return here


def test_unpack_quirks(orc):
    # an item is read only with 32 bytes left: a last item of 0..6 data bytes cannot be unpacked
    for n in range(0, 9):
        p = build([(1, 2, bytes(range(n)))])
        want = (7, 1, len(p), 0, 0) if n >= 7 else (5, 0, 64, 25 + n, 7 - n)
        assert orc.metadata_unpack(p) == want == py_unpack(p), n
    assert orc.metadata_unpack(build([])) == (7, 0, 64, 0, 0)          # no items: MD5("") checked
    p = build([(1, 2, b"0123456789")] * 3)
    assert orc.metadata_unpack(p[:-1]) == (6, 2, 2 * 35 + 64 + 24, 10, 1)   # last canary missing
    assert orc.metadata_unpack(p + b"xyz")[:2] == (7, 3)                # item_count stops the walk


# ---- GPU ----------------------------------------------------------------------------------------
def scatter(rng, packs):
    """Packs in one buffer at arbitrary byte offsets (gaps of 0..7 random bytes)."""
    offs, parts, pos = [], [], 0
    for p in packs:
        gap = rng.integers(0, 256, int(rng.integers(0, 8)), dtype=np.uint8).tobytes()
        parts += [gap, p]
        pos += len(gap)
        offs.append(pos)
        pos += len(p)
    buf = np.frombuffer(b"".join(parts) + b"\0", np.uint8).copy()
    return buf, np.array(offs, np.uint64), np.array([len(p) for p in packs], np.uint32)


def infos_as_tuples(info):
    return [tuple(int(x) for x in r) for r in info.tolist()]


@pytest.mark.gpu
@pytest.mark.parametrize("seg_line,slots", [(1, 3), (1, 2), (2, 0), (0, 0)])
def test_unpack_batch_vs_oracle(brb, orc, seg_line, slots):
    """seg_line 1: the line-staged kernel (round 4) with `slots` LDS-DMA ring slots (test option
    line_slots), 2: its producer / consumer wave-pair form, 0: the per-lane kernel."""
    packs = corpus(3, 4000)
    rng = np.random.default_rng(4)
    buf, offs, lens = scatter(rng, packs)
    want = [orc.metadata_unpack(p) for p in packs]
    with brb.TestOption("seg_line", seg_line), brb.TestOption("line_slots", slots):
        got = infos_as_tuples(brb.metadata_unpack_batch(buf, offs, lens))      # host mode
        assert got == want
        import torch
        d = torch.from_numpy(buf).cuda()
        o = torch.from_numpy(offs.view(np.int64)).cuda()
        ln = torch.from_numpy(lens.view(np.int32)).cuda()
        dev = brb.metadata_unpack_batch(d, o, ln).cpu().numpy().reshape(-1).view(brb.METADATA_INFO_DTYPE)
        assert infos_as_tuples(dev) == want
        assert infos_as_tuples(brb.metadata_unpack_batch(buf, offs, lens, all_devices=True)) == want


@pytest.mark.gpu
@pytest.mark.parametrize("seg_line", [1, 2, 0])
def test_unpack_batch_bench_count(brb, orc, seg_line):
    """A bench-sized batch: 65 536 valid and mutated packs (every return code) at arbitrary byte
    offsets, device mode, every BRB_MetaDataUnpackInfo field against the oracle."""
    import torch
    packs = corpus(7, 65536)
    buf, offs, lens = scatter(np.random.default_rng(8), packs)
    want = [orc.metadata_unpack(p) for p in packs]
    d = torch.from_numpy(buf).cuda()
    o = torch.from_numpy(offs.view(np.int64)).cuda()
    ln = torch.from_numpy(lens.view(np.int32)).cuda()
    with brb.TestOption("seg_line", seg_line):
        dev = brb.metadata_unpack_batch(d, o, ln).cpu().numpy().reshape(-1).view(brb.METADATA_INFO_DTYPE)
    assert infos_as_tuples(dev) == want
    assert len({w[0] for w in want}) >= 5                     # the corpus reaches the return codes


@pytest.mark.gpu
@pytest.mark.parametrize("seg_line", [1, 2])
def test_unpack_many_groups_per_wave(brb, orc, seg_line):
    """More groups than the launch has waves (line kernel) or wave pairs (pair kernel): 200 000
    packs = 3 125 groups on at most 1 024, three or four groups in sequence per wave / pair.  The
    packs are 3 000 corpus packs repeated at scattered offsets; the whole buffer is copied a second
    time past 2 GiB, and one pack of every fifth group is read from that copy, so those groups take
    the per-lane path (the producer alone) between planned ones.  Every field vs the oracle."""
    import torch
    uniq = corpus(29, 3000)
    want_u = [orc.metadata_unpack(p) for p in uniq]
    n = 200_000
    idx = np.random.default_rng(30).integers(0, len(uniq), n)
    buf, offs, lens = scatter(np.random.default_rng(31), [uniq[i] for i in idx])
    far = (1 << 31) + 777
    d = torch.zeros(far + buf.size, dtype=torch.uint8, device="cuda")
    src = torch.from_numpy(buf).cuda()
    d[: buf.size] = src
    d[far:] = src
    groups = (n + 63) // 64
    wide = [64 * g + 9 for g in range(2, groups, 5)]
    offs[wide] += np.uint64(far)
    o = torch.from_numpy(offs.view(np.int64)).cuda()
    ln = torch.from_numpy(lens.view(np.int32)).cuda()
    with brb.TestOption("seg_line", seg_line):
        dev = brb.metadata_unpack_batch(d, o, ln).cpu().numpy().reshape(-1).view(brb.METADATA_INFO_DTYPE)
    assert infos_as_tuples(dev) == [want_u[i] for i in idx]
    del d, src
    torch.cuda.empty_cache()


@pytest.mark.gpu
@pytest.mark.parametrize("seg_line", [1, 2])
@pytest.mark.parametrize("n_items,item_len,gap", [(4, 375, 0), (9, 61, 3), (40, 2, 1), (2, 1000, 77), (13, 0, 5)])
def test_unpack_uniform_layouts(brb, orc, n_items, item_len, gap, seg_line):
    """Batches whose packs share one layout (the bench's 4 x 375-byte items, and tiny / empty /
    large items), so every lane of a wave reaches its events in the same line; packs back to back
    or with `gap` bytes between them; 20 % carry a flipped byte; every field vs the oracle."""
    rng = np.random.default_rng(n_items * 1000 + item_len)
    packs = []
    for i in range(5000):
        items = [(j, i, rng.integers(0, 256, item_len, dtype=np.uint8).tobytes()) for j in range(n_items)]
        p = bytearray(build(items))
        if rng.random() < 0.2:
            p[int(rng.integers(0, len(p)))] ^= 1 << int(rng.integers(0, 8))
        packs.append(bytes(p))
    parts, offs, pos = [], [], 0
    for p in packs:
        offs.append(pos)
        parts.append(p + bytes(gap))
        pos += len(p) + gap
    buf = np.frombuffer(b"".join(parts) + b"\0", np.uint8).copy()
    lens = np.array([len(p) for p in packs], np.uint32)
    with brb.TestOption("seg_line", seg_line):
        got = infos_as_tuples(brb.metadata_unpack_batch(buf, np.array(offs, np.uint64), lens))
    assert got == [orc.metadata_unpack(p) for p in packs]


@pytest.mark.gpu
def test_unpack_pair_fault_reported(brb, orc):
    """A protocol fault in the MetaData producer / consumer pair (test option pair_stall: the first
    pair never posts its first plan) makes the call fail with BRB_BATCH_FAULT (-4, pair_fault.h)
    instead of returning unpack results; the next call on the same thread is clean and exact."""
    rng = np.random.default_rng(37)
    packs = [build([(j, i, rng.integers(0, 256, 700, dtype=np.uint8).tobytes()) for j in range(3)])
             for i in range(300)]                         # > 46 ring words per lane: the producer blocks
    buf, offs, lens = scatter(rng, packs)
    with brb.TestOption("seg_line", 2), brb.TestOption("pair_stall", 1):
        with pytest.raises(RuntimeError, match=r"returned -4: wave-pair protocol fault"):
            brb.metadata_unpack_batch(buf, offs, lens)
    with brb.TestOption("seg_line", 2):
        got = infos_as_tuples(brb.metadata_unpack_batch(buf, offs, lens))
    assert got == [orc.metadata_unpack(p) for p in packs]
    assert {g[0] for g in got} == {7}


@pytest.mark.gpu
def test_pack_batch_round_trip(brb, orc):
    from brb_framework_amd import metadata
    rng = np.random.default_rng(5)
    packs = [random_items(rng, max_items=12, max_len=3000) for _ in range(600)] + [[], [(7, 8, b"")]]
    buf, offs, lens = metadata.pack_batch(packs)
    info = metadata.unpack_batch(buf, offs, lens)
    for p, items in enumerate(packs):
        raw = buf[int(offs[p]):int(offs[p]) + int(lens[p])].tobytes()
        assert raw == orc.metadata_pack(items)                                   # digest and layout
        assert tuple(int(x) for x in info[p].tolist()) == orc.metadata_unpack(raw)
        if info[p]["error_code"] == metadata.UNPACK_SUCCESS:
            assert metadata.items(raw) == items


@pytest.mark.gpu
@pytest.mark.parametrize("seg_line", [1, 2, 0])
def test_unpack_large_items(brb, orc, seg_line):
    """Items of 64 KiB .. 1 MiB (many MD5 blocks per lane, items spanning block boundaries at every
    byte offset) next to tiny packs in the same batch."""
    rng = np.random.default_rng(6)
    packs = []
    for n in (65536, 65537, 1 << 20, 3):
        items = [(1, 1, rng.integers(0, 256, n, dtype=np.uint8).tobytes()), (2, 2, b"x" * 13)]
        p = build(items)
        packs += [p, mutate(rng, items, p)]
    buf, offs, lens = scatter(rng, packs)
    with brb.TestOption("seg_line", seg_line):
        got = infos_as_tuples(brb.metadata_unpack_batch(buf, offs, lens))
    assert got == [orc.metadata_unpack(p) for p in packs]


@pytest.mark.gpu
@pytest.mark.parametrize("seg_line", [1, 2])
def test_unpack_long_stretches(brb, orc, seg_line):
    """Work that outlasts a wait without progress: (1) a pack of 300 000 empty items (8 MB, tens of
    thousands of lines in which the walk emits no message word) beside ordinary packs, (2) a 64 MiB
    item in a pack placed more than 2 GiB from its group's other packs (the per-lane path, the
    producer alone while its partner waits for the next plan), and (3) the empty-item pack again on
    that per-lane path, where an empty item runs no block (the walk beats once per item).
    Every field vs the oracle."""
    import torch
    rng = np.random.default_rng(23)
    empty = build([(i & 0xFF, 1, b"") for i in range(300_000)])
    small = [build([(1, 2, rng.integers(0, 256, 300, dtype=np.uint8).tobytes())]) for _ in range(70)]
    huge = build([(3, 4, rng.integers(0, 256, 64 << 20, dtype=np.uint8).tobytes())])
    packs = [empty] + small[:63] + [huge, empty] + small[63:]
    far = (1 << 31) + 12345
    total = far + len(huge) + 8 + len(empty) + 64
    d = torch.zeros(total, dtype=torch.uint8, device="cuda")
    offs, pos = [], 0
    for i, p in enumerate(packs):
        if i == 64:
            o = far
        elif i == 65:
            o = far + len(huge) + 8
        else:
            o = pos
            pos += len(p) + 3
        offs.append(o)
        d[o:o + len(p)] = torch.from_numpy(np.frombuffer(p, np.uint8).copy()).cuda()
    assert pos < far
    offs = np.array(offs, np.uint64)
    lens = np.array([len(p) for p in packs], np.uint32)
    o = torch.from_numpy(offs.view(np.int64)).cuda()
    ln = torch.from_numpy(lens.view(np.int32)).cuda()
    with brb.TestOption("seg_line", seg_line):
        dev = brb.metadata_unpack_batch(d, o, ln).cpu().numpy().reshape(-1).view(brb.METADATA_INFO_DTYPE)
    want = [orc.metadata_unpack(p) for p in packs]
    assert infos_as_tuples(dev) == want
    assert want[64][0] == 7                                # the 64 MiB item unpacks (METADATA_UNPACK_SUCCESS)
    assert want[65] == want[0]
    assert want[0][1] == 299_999                           # every empty item walked; the last one is the
    #                                                        reference's < 32-bytes-left quirk (NEED_MORE_DATA_METAITEM)
    del d
    torch.cuda.empty_cache()


@pytest.mark.gpu
@pytest.mark.parametrize("seg_line", [1, 2])
def test_unpack_beyond_4gib(brb, orc, seg_line):
    """Packs at byte offsets past 2^32: the same 2 000 scattered packs copied into one 4.5 GiB
    device buffer three times -- straddling 2^31, straddling 2^32, and ending at the buffer's last
    byte -- and unpacked in one call; every BRB_MetaDataUnpackInfo field equals the oracle's."""
    import torch
    packs = corpus(13, 2000)
    buf, offs, lens = scatter(np.random.default_rng(14), packs)
    want = [orc.metadata_unpack(p) for p in packs]
    total = 9 << 29
    size = buf.size - 1                           # scatter() appends one NUL
    bases = [(1 << 31) - size // 2, (1 << 32) - size // 2, total - size]
    assert bases[0] + size <= bases[1] and bases[1] + size <= bases[2] and bases[2] + size == total
    d = torch.zeros(total, dtype=torch.uint8, device="cuda")
    src = torch.from_numpy(buf[:size].copy()).cuda()
    for b in bases:
        d[b:b + size] = src
    all_offs = np.concatenate([offs + np.uint64(b) for b in bases])
    all_lens = np.concatenate([lens] * 3)
    assert int((all_offs + all_lens).max()) <= total
    o = torch.from_numpy(all_offs.view(np.int64)).cuda()
    ln = torch.from_numpy(all_lens.view(np.int32)).cuda()
    with brb.TestOption("seg_line", seg_line):
        dev = brb.metadata_unpack_batch(d, o, ln).cpu().numpy().reshape(-1).view(brb.METADATA_INFO_DTYPE)
    assert infos_as_tuples(dev) == want * 3
    del d, src
    torch.cuda.empty_cache()
