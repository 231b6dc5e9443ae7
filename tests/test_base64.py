"""base64: the oracle against RFC 4648 and Python's base64 (CPU), and the GPU
batches (BRB_Base64EncodeBatch / BRB_Base64DecodeBatch) against the oracle, bit for bit."""
import base64

import numpy as np
import pytest

from brb_framework_amd import workload

RFC4648 = [(b"", b""), (b"f", b"Zg=="), (b"fo", b"Zm8="), (b"foo", b"Zm9v"), (b"foob", b"Zm9vYg=="),
           (b"fooba", b"Zm9vYmE="), (b"foobar", b"Zm9vYmFy")]


def test_oracle_rfc4648(orc):
    for plain, enc in RFC4648:
        assert orc.b64_encode(plain) == enc
        # the reference counts '=' as the value 0 (base64.c:374): padding decodes to zero bytes
        assert orc.b64_decode(enc) == plain + b"\0" * enc.count(b"=")


def test_oracle_vs_python(orc):
    rng = np.random.default_rng(4)
    for _ in range(200):
        data = rng.integers(0, 256, int(rng.integers(0, 400)), dtype=np.uint8).tobytes()
        enc = orc.b64_encode(data)
        assert enc == base64.b64encode(data)
        assert orc.b64_decode(enc) == data + b"\0" * enc.count(b"=")
        # noise outside the alphabet is skipped (base64.c:143-144); a NUL ends the string
        noisy = b"".join(bytes([c]) + (b"\n" if i % 7 == 0 else b"") for i, c in enumerate(enc))
        assert orc.b64_decode(noisy) == orc.b64_decode(enc)
        assert orc.b64_decode(enc[:8] + b"\0" + enc[8:]) == orc.b64_decode(enc[:8])


@pytest.fixture(scope="module")
def torch_dev(brb):
    import torch
    assert torch.cuda.is_available(), "no HIP device visible to torch"
    assert brb.gpu_available(), brb.lib().BRB_CryptoGPU_LastError()
    return torch


def _records(seed, n, max_len):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, max_len + 1, n).astype(np.uint32)
    lens[: min(n, 30)] = np.arange(min(n, 30))
    offs, pos = [], 3
    for L in lens:
        pos += int(rng.integers(0, 4))
        offs.append(pos)
        pos += int(L)
    return workload.gen_records(0x5EED00B6 + seed, 0, 1, pos + 8), np.array(offs, np.uint64), lens


@pytest.mark.gpu
@pytest.mark.parametrize("group", [-1, 0, 1, 3, 4, 5, 6])
@pytest.mark.parametrize("seed,n,max_len", [(1, 500, 40), (2, 300, 3000), (3, 20, 100000)])
def test_encode_decode_batch(brb, orc, torch_dev, seed, n, max_len, group):
    """group: log2 of the lanes per record (test option b64_group; -1 = the launcher's choice, from
    the mean length in host mode and 32 lanes in device mode).
    Records start and end at every byte alignment, inputs and outputs alike."""
    with brb.TestOption("b64_group", group):
        _encode_decode_batch(brb, orc, torch_dev, seed, n, max_len)


def _encode_decode_batch(brb, orc, torch_dev, seed, n, max_len):
    data, offs, lens = _records(seed, n, max_len)
    want = [orc.b64_encode(data[int(o):int(o) + int(L)].tobytes()) for o, L in zip(offs, lens)]
    elens = np.array([len(w) for w in want], np.uint32)
    eoffs = np.zeros(n, np.uint64)
    eoffs[1:] = np.cumsum(elens.astype(np.uint64) + 1)[:-1]      # 1-byte gaps between outputs
    total = int(eoffs[-1] + elens[-1] + 8)
    # host mode
    out = np.full(total, 0xEE, np.uint8)
    brb.base64_encode_batch(data, offs, lens, out, eoffs)
    for i in range(n):
        assert out[int(eoffs[i]):int(eoffs[i]) + int(elens[i])].tobytes() == want[i]
        assert out[int(eoffs[i]) + int(elens[i])] == 0xEE                  # nothing past the record
    # device mode
    t = torch_dev
    dout = t.full((total,), 0xEE, dtype=t.uint8, device="cuda")
    brb.base64_encode_batch(t.from_numpy(data).cuda(), t.from_numpy(offs).cuda(), t.from_numpy(lens).cuda(), dout,
                            t.from_numpy(eoffs).cuda())
    assert np.array_equal(dout.cpu().numpy(), out)
    # decode the encodings back (with noise bytes and an early NUL in some records)
    text = out.copy()
    for i in range(0, n, 5):
        if elens[i] > 6:
            text[int(eoffs[i]) + 3] = ord("\n")                 # skipped
    for i in range(2, n, 11):
        if elens[i] > 10:
            text[int(eoffs[i]) + 9] = 0                           # ends the C string
    dlen_cap = 3 * (elens // 4)
    doffs = np.zeros(n, np.uint64)
    doffs[1:] = np.cumsum(dlen_cap.astype(np.uint64))[:-1]
    dtotal = int(dlen_cap.sum()) + 8
    hout = np.zeros(dtotal, np.uint8)
    got_len = brb.base64_decode_batch(text, eoffs, elens, hout, doffs)
    dd = t.zeros(dtotal, dtype=t.uint8, device="cuda")
    dl = brb.base64_decode_batch(t.from_numpy(text).cuda(), t.from_numpy(eoffs).cuda(), t.from_numpy(elens).cuda(),
                                 dd, t.from_numpy(doffs).cuda())
    dd = dd.cpu().numpy()
    dl = dl.cpu().numpy()
    for i in range(n):
        rec = text[int(eoffs[i]):int(eoffs[i]) + int(elens[i])].tobytes()
        w = orc.b64_decode(rec)
        assert int(got_len[i]) == len(w) and int(dl[i]) == len(w), i
        assert hout[int(doffs[i]):int(doffs[i]) + len(w)].tobytes() == w
        assert dd[int(doffs[i]):int(doffs[i]) + len(w)].tobytes() == w


@pytest.mark.gpu
@pytest.mark.parametrize("group", [-1, 0, 2, 5, 6])
def test_decode_falls_back_mid_record(brb, orc, group):
    """Long records whose first skipped byte, NUL or '=' run comes after many fixed-position pieces:
    the pieces' output and the serial remainder must join exactly (base64.c:131-179), and nothing is
    written past the decoded bytes."""
    with brb.TestOption("b64_group", group):
        _decode_falls_back_mid_record(brb, orc)


def _decode_falls_back_mid_record(brb, orc):
    rng = np.random.default_rng(9)
    n = 400
    texts = []
    for i in range(n):
        plain = rng.integers(0, 256, int(rng.integers(300, 3000)), dtype=np.uint8).tobytes()
        t = bytearray(orc.b64_encode(plain))
        kind = i % 5
        at = int(rng.integers(0, len(t)))
        if kind == 1:
            t[at] = ord("\n")                                   # skipped: the groups after it shift by one
        elif kind == 2:
            t[at] = 0                                           # ends the C string
        elif kind == 3:
            t[at:at] = b"*#\r"                                  # three skipped bytes
        elif kind == 4:
            t[at] = ord("=")                                    # counts as the value 0
        texts.append(bytes(t))
    lens = np.array([len(t) for t in texts], np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens.astype(np.uint64) + 3)[:-1]          # 3-byte gaps: every alignment
    buf = np.zeros(int(offs[-1]) + int(lens[-1]) + 8, np.uint8)
    for o, t in zip(offs, texts):
        buf[int(o):int(o) + len(t)] = np.frombuffer(t, np.uint8)
    cap = 3 * (lens // 4)
    doffs = np.zeros(n, np.uint64)
    doffs[1:] = np.cumsum(cap.astype(np.uint64) + 1)[:-1]
    out = np.full(int(cap.sum()) + n + 8, 0xEE, np.uint8)
    got = brb.base64_decode_batch(buf, offs, lens, out, doffs)
    for i, t in enumerate(texts):
        w = orc.b64_decode(t)
        assert int(got[i]) == len(w), i
        assert out[int(doffs[i]):int(doffs[i]) + len(w)].tobytes() == w, i
        assert out[int(doffs[i]) + len(w)] == 0xEE, i             # nothing written past the decoded bytes


@pytest.mark.gpu
def test_full_shape_round_trip(brb, torch_dev):
    """The f4 bench shape at full size: 65 536 records x 1500 B encoded on the GPU equal Python's
    base64 (RFC 4648) on every record, and decode back to the records (1500 bytes each)."""
    t = torch_dev
    n, L = 65536, 1500
    T = 4 * ((L + 2) // 3)
    data = workload.gen_records(0x5EED00B6, 0, n, L)
    offs = np.arange(n, dtype=np.uint64) * L
    lens = np.full(n, L, np.uint32)
    toffs = np.arange(n, dtype=np.uint64) * T
    tlens = np.full(n, T, np.uint32)
    text = t.zeros(n * T, dtype=t.uint8, device="cuda")
    brb.base64_encode_batch(t.from_numpy(data).cuda(), t.from_numpy(offs).cuda(), t.from_numpy(lens).cuda(), text,
                            t.from_numpy(toffs).cuda())
    got = text.cpu().numpy().reshape(n, T)
    want = np.frombuffer(b"".join(base64.b64encode(data[i * L:(i + 1) * L].tobytes()) for i in range(n)),
                         np.uint8).reshape(n, T)
    assert np.array_equal(got, want)
    back = t.zeros(n * L, dtype=t.uint8, device="cuda")
    olens = brb.base64_decode_batch(text, t.from_numpy(toffs).cuda(), t.from_numpy(tlens).cuda(), back,
                                    t.from_numpy(offs).cuda())
    assert (olens.cpu().numpy() == L).all()
    assert np.array_equal(back.cpu().numpy(), data)


@pytest.mark.gpu
@pytest.mark.parametrize("group", [-1, 0, 3, 5, 6])
def test_group_kernels_fuzz(brb, orc, torch_dev, group):
    """Many small batches of mixed lengths through the group kernels (test option b64_group): the
    piece boundaries of encode (12 bytes) and decode (16 characters) against every tail length,
    records of 0..200 bytes mixed with a few long ones in one group, every input and output byte
    alignment, device and host mode; bytes between the outputs stay untouched."""
    rng = np.random.default_rng(77 + group)
    t = torch_dev
    with brb.TestOption("b64_group", group):
        for trial in range(6):
            n = int(rng.integers(1, 300))
            lens = rng.integers(0, 200, n).astype(np.uint32)
            lens[rng.integers(0, n, max(1, n // 30))] = rng.integers(1000, 5000, max(1, n // 30))
            offs = np.zeros(n, np.uint64)
            pos = int(rng.integers(0, 4))
            for i in range(n):
                offs[i] = pos
                pos += int(lens[i]) + int(rng.integers(0, 5))
            data = rng.integers(0, 256, pos + 8, dtype=np.uint8)
            want = [orc.b64_encode(data[int(o):int(o) + int(L)].tobytes()) for o, L in zip(offs, lens)]
            elens = np.array([len(w) for w in want], np.uint32)
            eoffs = np.zeros(n, np.uint64)
            p = int(rng.integers(0, 4))
            for i in range(n):
                eoffs[i] = p
                p += int(elens[i]) + 1 + int(rng.integers(0, 3))
            total = p + 8
            dev = trial % 2 == 1
            if dev:
                o = t.full((total,), 0xA5, dtype=t.uint8, device="cuda")
                brb.base64_encode_batch(t.from_numpy(data).cuda(), t.from_numpy(offs).cuda(), t.from_numpy(lens).cuda(),
                                        o, t.from_numpy(eoffs).cuda())
                out = o.cpu().numpy()
            else:
                out = np.full(total, 0xA5, np.uint8)
                brb.base64_encode_batch(data, offs, lens, out, eoffs)
            mask = np.ones(total, bool)
            for i in range(n):
                a, L = int(eoffs[i]), int(elens[i])
                assert out[a:a + L].tobytes() == want[i], (trial, i, int(lens[i]))
                mask[a:a + L] = False
            assert (out[mask] == 0xA5).all()
            # decode back, with a few skipped bytes / NULs planted in some records
            text = out.copy()
            for i in rng.integers(0, n, max(1, n // 10)):
                if elens[i] > 2:
                    text[int(eoffs[i]) + int(rng.integers(0, elens[i]))] = int(rng.choice([0, 10, 33, 61]))
            cap = 3 * (elens // 4)
            doffs = np.zeros(n, np.uint64)
            q = int(rng.integers(0, 4))
            for i in range(n):
                doffs[i] = q
                q += int(cap[i]) + 1
            if dev:
                d = t.full((q + 8,), 0x5A, dtype=t.uint8, device="cuda")
                dl = brb.base64_decode_batch(t.from_numpy(text).cuda(), t.from_numpy(eoffs).cuda(),
                                             t.from_numpy(elens).cuda(), d, t.from_numpy(doffs).cuda())
                dec, dl = d.cpu().numpy(), dl.cpu().numpy()
            else:
                dec = np.full(q + 8, 0x5A, np.uint8)
                dl = brb.base64_decode_batch(text, eoffs, elens, dec, doffs)
            dmask = np.ones(q + 8, bool)
            for i in range(n):
                w = orc.b64_decode(text[int(eoffs[i]):int(eoffs[i]) + int(elens[i])].tobytes())
                assert int(dl[i]) == len(w), (trial, i)
                a = int(doffs[i])
                assert dec[a:a + len(w)].tobytes() == w, (trial, i)
                dmask[a:a + len(w)] = False
            assert (dec[dmask] == 0x5A).all()


@pytest.mark.gpu
def test_beyond_4gib(brb, orc, torch_dev):
    """Input offsets past 2^32 (encode) and output offsets past 2^32 (decode) in one 4.5 GiB device
    buffer: 300 records of 0..3000 bytes, some straddling byte offsets 2^31 and 2^32, encoded into
    a small text buffer (== Python's base64) and decoded back into the big buffer's top 8 MiB (==
    the oracle's decode, which keeps the reference's length rule: whole 3-byte groups)."""
    t = torch_dev
    total = 9 << 29
    words = t.empty(total // 8, dtype=t.int64, device="cuda")
    g = t.Generator(device="cuda")
    g.manual_seed(0x4B1D)
    words.random_(generator=g)
    d = words.view(t.uint8)
    rng = np.random.default_rng(21)
    n = 300
    lens = rng.integers(0, 3001, n).astype(np.uint32)
    offs = rng.integers(0, total - (16 << 20), n).astype(np.uint64)
    for i, o in enumerate([(1 << 31) - 1000, (1 << 32) - 1000, (1 << 32) - 1, (1 << 32) + 1]):
        offs[i], lens[i] = o, 2000
    host = [d[int(o):int(o) + int(m)].cpu().numpy().tobytes() for o, m in zip(offs, lens)]
    want = [base64.b64encode(h) for h in host]
    tl = np.array([len(w) for w in want], np.uint32)
    to = np.zeros(n, np.uint64)
    to[1:] = np.cumsum(tl.astype(np.uint64))[:-1]
    text = t.zeros(int(tl.sum()) + 8, dtype=t.uint8, device="cuda")
    dev = lambda a: t.from_numpy(np.ascontiguousarray(a)).cuda()   # noqa: E731
    brb.base64_encode_batch(d, dev(offs), dev(lens), text, dev(to))
    tx = text.cpu().numpy()
    for i in range(n):
        assert tx[int(to[i]):int(to[i]) + int(tl[i])].tobytes() == want[i], f"record {i} at {int(offs[i])}"
    dec = [orc.b64_decode(w) for w in want]
    dl = np.array([len(x) for x in dec], np.uint64)
    doffs = np.zeros(n, np.uint64)
    doffs[1:] = np.cumsum(dl)[:-1]
    doffs += total - (8 << 20)
    olens = brb.base64_decode_batch(text, dev(to), dev(tl), d, dev(doffs)).cpu().numpy()
    for i in range(n):
        assert int(olens[i]) == len(dec[i]) and dec[i][:len(host[i])] == host[i]
        o = int(doffs[i])
        assert d[o:o + len(dec[i])].cpu().numpy().tobytes() == dec[i], f"decoded record {i} at {o}"
    del words, d
    t.cuda.empty_cache()
