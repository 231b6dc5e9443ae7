"""Seeded random shapes through every device-mode batch entry point, each checked against the oracle
(or hashlib for the segment digests): record lengths and counts drawn from mixtures that hit the
kernels' branch points (empty records, records of at most 64 bytes, whole and partial lines, the
1 500-byte shape, several groups per wave), data pointers at every byte alignment, offsets out of
order, overlapping and with gaps, and the segment kernels under each `seg_line` form.  Sizes are kept
so the whole file runs in well under a minute on one MI355X; the fixed seeds make a failure
reproducible.  SURVEY §7 edge cases; the reference has no tests of its own for this path (§4).
"""
import hashlib
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# batch sizes scale with BRB_FUZZ_SCALE (tools/fuzz_soak.py --scale; 1 in the suite)
SCALE = max(1, int(os.environ.get("BRB_FUZZ_SCALE", "1")))


def _n(hi):
    return hi * SCALE


@pytest.fixture(scope="module")
def torch_dev(brb):
    import torch
    assert torch.cuda.is_available(), "no HIP device visible to torch"
    assert brb.gpu_available(), brb.lib().BRB_CryptoGPU_LastError()
    return torch


def _lengths(rng, n, hi=5000):
    """A mixture: empty, one block or less, around the 128-byte line, mid, long."""
    kind = rng.integers(0, 10, n)
    out = np.where(kind == 0, 0,
          np.where(kind <= 3, rng.integers(1, 65, n),
          np.where(kind == 4, rng.integers(100, 160, n),
          np.where(kind <= 8, rng.integers(160, min(1700, hi), n), rng.integers(min(1700, hi - 1), hi, n)))))
    return out.astype(np.uint32)


def _layout(rng, lens, overlap):
    """Offsets for records of `lens`: packed in a shuffled order with gaps of 0..7 bytes, or (overlap)
    anywhere in a buffer a little longer than the longest record."""
    n = len(lens)
    if overlap:
        size = int(lens.max(initial=0)) + int(rng.integers(1, 4096))
        offs = (rng.random(n) * (size - lens + 1)).astype(np.uint64)
        return offs, size
    order = rng.permutation(n)
    offs = np.zeros(n, np.uint64)
    pos = int(rng.integers(0, 16))
    for i in order:
        offs[i] = pos
        pos += int(lens[i]) + int(rng.integers(0, 8))
    return offs, pos + 16


def _dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("seed", range(12))
def test_fuzz_fixed_stride(brb, orc, torch_dev, seed):
    """BRB_MD5BatchFixed / BrbSha1_BatchFixed: random record length and count, the batch starting at
    any byte of a device buffer (line-staged, record-relative and 64-byte kernels alike)."""
    rng = np.random.default_rng(0xF1C5 + seed)
    for _ in range(6):
        pick = rng.integers(0, 4)
        rec_len = int([rng.integers(1, 130), rng.integers(130, 3100), rng.integers(3100, 9000),
                       rng.choice([63, 64, 65, 127, 128, 129, 1500, 2048])][pick])
        n = int(rng.integers(1, _n(3000) if rec_len < 3100 else _n(400)))
        shift = int(rng.integers(0, 64))
        data = rng.integers(0, 256, shift + rec_len * n + 64, dtype=np.uint8)
        d = _dev(torch_dev, data)
        sub = d[shift:shift + rec_len * n]
        host = np.ascontiguousarray(data[shift:shift + rec_len * n])
        got5 = brb.md5_batch_fixed(sub, rec_len, n).cpu().numpy()
        assert np.array_equal(got5, orc.md5_batch_fixed(host, rec_len, n, threads=8)), (rec_len, n, shift)
        got1 = brb.sha1_batch_fixed(sub, rec_len, n).cpu().numpy()
        assert np.array_equal(got1, orc.sha1_batch_fixed(host, rec_len, n, threads=8)), (rec_len, n, shift)


@pytest.mark.parametrize("seed", range(10))
def test_fuzz_variable_length(brb, orc, torch_dev, seed):
    """BRB_MD5Batch / BrbSha1_Batch: mixed lengths (empty records included), offsets out of order,
    with gaps or overlapping."""
    rng = np.random.default_rng(0xF2C5 + seed)
    for case in range(4):
        n = int(rng.integers(1, _n(2500)))
        lens = _lengths(rng, n)
        offs, size = _layout(rng, lens, overlap=bool(case & 1))
        data = rng.integers(0, 256, size, dtype=np.uint8)
        d, o, ln = _dev(torch_dev, data), _dev(torch_dev, offs.view(np.int64)), _dev(torch_dev, lens.view(np.int32))
        got5 = brb.md5_batch(d, o, ln).cpu().numpy()
        assert np.array_equal(got5, orc.md5_batch(data, offs, lens, threads=8)), (seed, case)
        got1 = brb.sha1_batch(d, o, ln).cpu().numpy()
        assert np.array_equal(got1, orc.sha1_batch(data, offs, lens, threads=8)), (seed, case)


@pytest.mark.parametrize("seg_line", [0, 1, 2])
@pytest.mark.parametrize("seed", range(5))
def test_fuzz_segments(brb, torch_dev, seed, seg_line):
    """BRB_MD5BatchSegments: 0..7 segments per record, empty ones included, anywhere in the buffer
    (overlapping), under each kernel form (seg_line 0 per-lane, 1 line-staged, 2 wave pairs)."""
    rng = np.random.default_rng(0xF3C5 + 16 * seed + seg_line)
    for _ in range(3):
        n = int(rng.integers(1, _n(1200)))
        k = rng.integers(0, 8, n)
        k[0] = max(int(k[0]), 1)                  # at least one segment in the call
        first = np.concatenate([[0], np.cumsum(k)]).astype(np.uint64)
        slens = _lengths(rng, int(first[-1]), hi=900)
        size = int(slens.max(initial=0)) + 8192
        soffs = (rng.random(len(slens)) * (size - slens + 1)).astype(np.uint64)
        data = rng.integers(0, 256, size, dtype=np.uint8)
        with brb.TestOption("seg_line", seg_line):
            got = brb.md5_batch_segments(_dev(torch_dev, data), _dev(torch_dev, soffs.view(np.int64)),
                                         _dev(torch_dev, slens.view(np.int32)),
                                         _dev(torch_dev, first.view(np.int64))).cpu().numpy()
        for r in range(n):
            h = hashlib.md5()
            for s in range(int(first[r]), int(first[r + 1])):
                h.update(data[int(soffs[s]):int(soffs[s]) + int(slens[s])].tobytes())
            assert got[r].tobytes() == h.digest(), (seed, seg_line, r)


@pytest.mark.parametrize("seed", range(10))
def test_fuzz_rc4(brb, orc, torch_dev, seed):
    """BRB_RC4_CryptBatch in place: mixed stream lengths at any byte offset, two passes so the
    states carry; ciphertext and states against the oracle."""
    rng = np.random.default_rng(0xF4C5 + seed)
    n = int(rng.integers(1, _n(1500)))
    lens = _lengths(rng, n, hi=3000)
    offs, size = _layout(rng, lens, overlap=False)
    data = rng.integers(0, 256, size, dtype=np.uint8)
    keys = [rng.integers(0, 256, int(rng.integers(1, 33)), dtype=np.uint8).tobytes() for _ in range(n)]
    st = brb.rc4_states(keys)
    want_data, want_st = data.copy(), st.copy()
    d, s = _dev(torch_dev, data), _dev(torch_dev, st)
    o, ln = _dev(torch_dev, offs.view(np.int64)), _dev(torch_dev, lens.view(np.int32))
    for _ in range(2):
        brb.rc4_crypt_batch(s, d, o, ln)
        orc.rc4_crypt_batch(want_st, want_data, offs, lens, threads=8)
    assert np.array_equal(d.cpu().numpy(), want_data)
    assert np.array_equal(s.cpu().numpy(), want_st)


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_base64(brb, orc, torch_dev, seed):
    """BRB_Base64EncodeBatch / DecodeBatch: mixed lengths (0 included) at any offset; the text against
    the oracle's encoder; decoded back as the reference decodes (each "=" a zero byte)."""
    rng = np.random.default_rng(0xF5C5 + seed)
    n = int(rng.integers(1, _n(400)))
    lens = _lengths(rng, n, hi=2500)
    offs, size = _layout(rng, lens, overlap=False)
    data = rng.integers(0, 256, size, dtype=np.uint8)
    tl = (4 * ((lens.astype(np.uint64) + 2) // 3)).astype(np.uint64)
    toffs = np.concatenate([[0], np.cumsum(tl + 3)[:-1]]).astype(np.uint64)
    text = _dev(torch_dev, np.zeros(int(toffs[-1] + tl[-1]) + 8, np.uint8))
    d = _dev(torch_dev, data)
    o, ln, to = (_dev(torch_dev, offs.view(np.int64)), _dev(torch_dev, lens.view(np.int32)),
                 _dev(torch_dev, toffs.view(np.int64)))
    brb.base64_encode_batch(d, o, ln, text, to)
    th = text.cpu().numpy()
    for i in range(n):
        want = orc.b64_encode(data[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes())
        assert th[int(toffs[i]):int(toffs[i]) + int(tl[i])].tobytes() == want, (seed, i)
    # decode back; the reference decodes each '=' as a zero byte (base64.c:374), so record i decodes
    # to its bytes plus one zero per '=': an output slot of 3 * len / 4 bytes and a guard byte
    dcap = (3 * (tl // 4)).astype(np.uint64)
    doffs = np.concatenate([[0], np.cumsum(dcap + 1)[:-1]]).astype(np.uint64)
    back = _dev(torch_dev, np.full(int(doffs[-1] + dcap[-1]) + 8, 0xEE, np.uint8))
    olen = brb.base64_decode_batch(text, to, _dev(torch_dev, tl.astype(np.uint32).view(np.int32)), back,
                                   _dev(torch_dev, doffs.view(np.int64))).cpu().numpy().astype(np.uint32)
    bh = back.cpu().numpy()
    for i in range(n):
        want = orc.b64_decode(th[int(toffs[i]):int(toffs[i]) + int(tl[i])].tobytes())
        a = int(doffs[i])
        assert int(olen[i]) == len(want), (seed, i)
        assert bh[a:a + len(want)].tobytes() == want, (seed, i)
        assert want[:int(lens[i])] == data[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes(), (seed, i)
        assert bh[a + len(want)] == 0xEE, (seed, i)                 # nothing past the decoded bytes


@pytest.mark.parametrize("seed", range(5))
def test_fuzz_blowfish(brb, orc, torch_dev, seed):
    """BRB_Blowfish_EncryptBatch / DecryptBatch: random block counts and 64-bit words (high halves
    set), random keys; ciphertext against the oracle, then the exact round trip."""
    rng = np.random.default_rng(0xF6C5 + seed)
    key = rng.integers(0, 256, int(rng.integers(1, 57)), dtype=np.uint8).tobytes()
    ctx = brb.blowfish_init(key)
    n = int(rng.integers(1, _n(200000)))
    words = rng.integers(0, 2**63, 2 * n, dtype=np.int64) * np.int64(1 + (seed & 1))
    w = _dev(torch_dev, words)
    brb.blowfish_encrypt_batch(ctx, w, n_blocks=n)
    want = orc.bf_ecb(orc.bf_init(key), words.view(np.uint64).copy(), threads=8)     # in place: a copy
    assert np.array_equal(w.cpu().numpy().view(np.uint64), want)
    brb.blowfish_decrypt_batch(ctx, w, n_blocks=n)
    assert np.array_equal(w.cpu().numpy(), words)


@pytest.mark.parametrize("seed", range(8))
def test_fuzz_rc4md5_frame_open(brb, orc, torch_dev, seed):
    """BRB_RC4MD5_FrameBatch then OpenBatch: mixed payload lengths (0 included) at any offset, frames
    at any offset, random salts; frames and states against the oracle; then a few frames damaged
    (one byte flipped) so their validation result is the oracle's (a flip inside the salt passes)."""
    rng = np.random.default_rng(0xF7C5 + seed)
    H = brb.RC4MD5_HEADER
    n = int(rng.integers(1, _n(1200)))
    lens = _lengths(rng, n, hi=3000)
    offs, size = _layout(rng, lens, overlap=False)
    payload = rng.integers(0, 256, size, dtype=np.uint8)
    flens = (lens + H).astype(np.uint32)
    foffs, fsize = _layout(rng, flens, overlap=False)
    salts = rng.integers(0, 2**32, n, dtype=np.uint64)
    keys = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(n)]
    st = brb.rc4_states(keys)
    wst, want_frames = st.copy(), np.zeros(fsize, np.uint8)
    orc.rc4md5_frame_batch(wst, payload, offs, lens, salts, want_frames, foffs, threads=8)
    dst = _dev(torch_dev, st)
    frames = _dev(torch_dev, np.zeros(fsize, np.uint8))
    fo = _dev(torch_dev, foffs.view(np.int64))
    brb.rc4md5_frame_batch(dst, _dev(torch_dev, payload), _dev(torch_dev, offs.view(np.int64)),
                           _dev(torch_dev, lens.view(np.int32)), _dev(torch_dev, salts.view(np.int64)), frames, fo)
    fh = frames.cpu().numpy()
    for i in range(n):
        a, b = int(foffs[i]), int(foffs[i]) + int(flens[i])
        assert fh[a:b].tobytes() == want_frames[a:b].tobytes(), (seed, i)
    assert np.array_equal(dst.cpu().numpy(), wst)
    bad = rng.choice(n, size=min(n, 5), replace=False)
    for i in bad:
        fh[int(foffs[i]) + int(rng.integers(0, int(flens[i])))] ^= 0x20
    rst, want_open, want_valid = st.copy(), fh.copy(), np.zeros(n, np.uint8)
    orc.rc4md5_open_batch(rst, want_open, foffs, flens, want_valid, threads=8)
    drst, dfr = _dev(torch_dev, st), _dev(torch_dev, fh)
    _, valid = brb.rc4md5_open_batch(drst, dfr, fo, _dev(torch_dev, flens.view(np.int32)))
    assert np.array_equal(valid.cpu().numpy().astype(np.uint8), want_valid)
    good = np.setdiff1d(np.arange(n), bad)
    assert (want_valid[good] == 1).all()        # a flipped salt byte is not checked: only the rest must be valid
    oh = dfr.cpu().numpy()
    for i in range(n):
        a, b = int(foffs[i]), int(foffs[i]) + int(flens[i])
        assert oh[a:b].tobytes() == want_open[a:b].tobytes(), (seed, i)
        if i not in bad:
            assert oh[a + H:b].tobytes() == payload[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes()
    assert np.array_equal(drst.cpu().numpy(), rst)


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_host_mode(brb, orc, torch_dev, seed):
    """The same shapes through host mode (numpy in and out: the library stages the records, runs the
    kernels and copies the results back): fixed and variable-length digests, segments, RC4."""
    rng = np.random.default_rng(0xF8C5 + seed)
    n = int(rng.integers(1, _n(2000)))
    lens = _lengths(rng, n)
    offs, size = _layout(rng, lens, overlap=bool(seed & 1))
    data = rng.integers(0, 256, size, dtype=np.uint8)
    assert np.array_equal(brb.md5_batch(data, offs, lens), orc.md5_batch(data, offs, lens, threads=8))
    assert np.array_equal(brb.sha1_batch(data, offs, lens), orc.sha1_batch(data, offs, lens, threads=8))
    rec_len = int(rng.integers(1, 3000))
    m = size // rec_len
    if m:
        fixed = np.ascontiguousarray(data[:rec_len * m])
        assert np.array_equal(brb.md5_batch_fixed(fixed, rec_len, m), orc.md5_batch_fixed(fixed, rec_len, m, threads=8))
    k = rng.integers(1, 5, n)
    first = np.concatenate([[0], np.cumsum(k)]).astype(np.uint64)
    slens = _lengths(rng, int(first[-1]), hi=900)
    soffs = (rng.random(len(slens)) * (size - np.minimum(slens, size) + 1)).astype(np.uint64)
    slens = np.minimum(slens, (size - soffs).astype(np.uint32))
    got = brb.md5_batch_segments(data, soffs, slens, first)
    for r in range(0, n, max(1, n // 200)):
        h = hashlib.md5()
        for s in range(int(first[r]), int(first[r + 1])):
            h.update(data[int(soffs[s]):int(soffs[s]) + int(slens[s])].tobytes())
        assert got[r].tobytes() == h.digest(), (seed, r)
    if not seed & 1:                              # RC4 in place needs streams that do not overlap
        st = brb.rc4_states([bytes([i & 255, (i >> 8) & 255, seed & 255]) for i in range(n)])
        want_d, want_st = data.copy(), st.copy()
        brb.rc4_crypt_batch(st, data, offs, lens)
        orc.rc4_crypt_batch(want_st, want_d, offs, lens, threads=8)
        assert np.array_equal(data, want_d) and np.array_equal(st, want_st)
