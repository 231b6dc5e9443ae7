"""RC4 and the RC4+MD5 frame of the comm transform.

CPU (not gpu): the oracle against the published RC4 vectors and OpenSSL, the compat BRB_RC4_* of
the product library against the oracle, and the frame fixtures (tests/golden/rc4.json).
GPU: BRB_RC4_CryptBatch / BRB_RC4MD5_FrameBatch / BRB_RC4MD5_OpenBatch through the C ABI against
the oracle, bit for bit, on ragged, misaligned and back-to-back streams, in host and device mode.
"""
import ctypes
import hashlib

import numpy as np
import pytest

from brb_framework_amd import workload

SEED = 0x5EED00F1


def _libcrypto():
    try:
        return ctypes.CDLL("libcrypto.so.3")
    except OSError:
        return None


# ---------------------------------------------------------------------------------------------
# CPU: oracle and compat surface
# ---------------------------------------------------------------------------------------------
def test_oracle_rc4_kat(orc, golden):
    for v in golden["rc4"]["kat"]:
        st = orc.rc4_init(bytes.fromhex(v["key"]))
        assert orc.rc4_crypt(st, bytes.fromhex(v["plain"]))[1].hex() == v["cipher"]


def test_oracle_rc4_vs_openssl(orc):
    L = _libcrypto()
    if L is None:
        pytest.skip("libcrypto.so.3 not present")
    rng = np.random.default_rng(11)
    for _ in range(30):
        key = rng.integers(0, 256, int(rng.integers(1, 257)), dtype=np.uint8).tobytes()
        data = rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes()
        ks = ctypes.create_string_buffer(2048)
        L.RC4_set_key(ks, len(key), key)
        out = ctypes.create_string_buffer(max(len(data), 1))
        L.RC4(ks, ctypes.c_size_t(len(data)), data, out)
        assert orc.rc4_crypt(orc.rc4_init(key), data)[1] == out.raw[: len(data)]


def test_oracle_streams_carry_state(orc, golden):
    for v in golden["rc4"]["streams"]:
        st = orc.rc4_init(bytes.fromhex(v["key"]))
        data, pos = bytes.fromhex(v["data"]), 0
        for n, want in zip(v["lens"], v["out"]):
            st, o = orc.rc4_crypt(st, data[pos:pos + n])
            assert o.hex() == want
            pos += n
        assert st.hex() == v["state_after"]


def test_oracle_frames(orc, golden):
    for v in golden["rc4"]["frames"]:
        st0 = orc.rc4_init(bytes.fromhex(v["key"]))
        payload = bytes.fromhex(v["payload"])
        st_w, fr = orc.rc4md5_frame(st0, payload, v["salt"])
        assert fr.hex() == v["frame"] and st_w.hex() == v["state_after"]
        st_r, dec, ok = orc.rc4md5_open(st0, fr)
        assert ok == 1 and dec[30:] == payload and dec[8:13] == b"HASH:"
        assert dec[13:29] == hashlib.md5(payload).digest() and dec[29] == 0
        assert int.from_bytes(dec[:8], "little") == v["salt"]


def test_oracle_open_rejects(orc):
    st0 = orc.rc4_init(b"cryptokey")
    _, fr = orc.rc4md5_frame(st0, b"payload bytes", 7)
    for pos in (8, 12, 13, 28, 30, len(fr) - 1):
        bad = bytearray(fr)
        bad[pos] ^= 1
        assert orc.rc4md5_open(st0, bytes(bad))[2] == 0, pos
    for pos in (0, 7, 29):       # salt and NUL are not checked (ev_kq_aio_transform.c:167-181)
        bad = bytearray(fr)
        bad[pos] ^= 1
        assert orc.rc4md5_open(st0, bytes(bad))[2] == 1, pos
    assert orc.rc4md5_open(st0, fr[:29])[2] == 0


def test_compat_rc4_matches_oracle(brb, orc, golden):
    for v in golden["rc4"]["kat"]:
        key, pt = bytes.fromhex(v["key"]), bytes.fromhex(v["plain"])
        st = brb.rc4_init(key)
        assert brb.rc4_state_bytes(st) == orc.rc4_init(key)
        out = ctypes.create_string_buffer(len(pt))
        brb.lib().BRB_RC4_Crypt(ctypes.byref(st), pt, out, len(pt))
        assert out.raw.hex() == v["cipher"]
    rng = np.random.default_rng(3)
    for _ in range(20):
        key = rng.integers(0, 256, int(rng.integers(1, 300)), dtype=np.uint8).tobytes()
        st, ost = brb.rc4_init(key), orc.rc4_init(key)
        for _ in range(3):          # the state carries across calls
            data = rng.integers(0, 256, int(rng.integers(0, 700)), dtype=np.uint8).tobytes()
            buf = ctypes.create_string_buffer(data, max(len(data), 1))
            brb.lib().BRB_RC4_Crypt(ctypes.byref(st), buf, buf, len(data))     # in place
            ost, want = orc.rc4_crypt(ost, data)
            assert buf.raw[: len(data)] == want and brb.rc4_state_bytes(st) == ost


def test_rc4_state_layout(brb):
    st = brb.BRB_RC4_State()
    assert ctypes.sizeof(st) == 264
    assert brb.BRB_RC4_State.index1.offset == 256 and brb.BRB_RC4_State.index2.offset == 257


# ---------------------------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def torch_dev(brb):
    import torch
    assert torch.cuda.is_available(), "no HIP device visible to torch"
    assert brb.gpu_available(), brb.lib().BRB_CryptoGPU_LastError()
    return torch


def _keys(n, seed=1):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 256, int(rng.integers(1, 64)), dtype=np.uint8).tobytes() for _ in range(n)]


def _layout(lens, gap_seed=None, base=0):
    """Back-to-back stream offsets (optionally with random 0..5-byte gaps) starting at `base`."""
    rng = np.random.default_rng(gap_seed) if gap_seed is not None else None
    offs, pos = [], base
    for n in lens:
        if rng is not None:
            pos += int(rng.integers(0, 6))
        offs.append(pos)
        pos += int(n)
    return np.array(offs, np.uint64), np.array(lens, np.uint32), pos


def _oracle_crypt(orc, states, data, offs, lens):
    out = data.copy()
    st = states.copy()
    for i, (o, n) in enumerate(zip(offs.tolist(), lens.tolist())):
        s2, ob = orc.rc4_crypt(st[i].tobytes(), data[o:o + n].tobytes())
        st[i] = np.frombuffer(s2, np.uint8)
        out[o:o + n] = np.frombuffer(ob, np.uint8)
    return st, out


def _to(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


RAGGED = [0, 1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 29, 30, 31, 32, 33, 63, 64, 65, 100, 255, 256, 257, 1000, 1500, 4099]


@pytest.fixture(params=[1, 0], ids=["pair", "single"])
def rc4_pair(request, brb):
    """Test option rc4_pair: 1 the keystream + I/O wave-pair RC4 pass (default), 0 one wave per stream."""
    with brb.TestOption("rc4_pair", request.param):
        yield request.param


@pytest.mark.gpu
@pytest.mark.parametrize("gaps", [None, 5])
@pytest.mark.parametrize("base", [0, 1, 2, 3])
def test_rc4_crypt_batch_ragged(brb, orc, torch_dev, gaps, base, rc4_pair):
    lens = (RAGGED * 5)[: 130]
    offs, lens, total = _layout(lens, gaps, base)
    data = workload.gen_records(SEED, base, 1, total + 8)
    states = brb.rc4_states(_keys(len(offs)))
    want_st, want = _oracle_crypt(orc, states, data, offs, lens)
    # device mode, in place
    t = _to(torch_dev, data)
    ts = _to(torch_dev, states)
    brb.rc4_crypt_batch(ts, t, _to(torch_dev, offs), _to(torch_dev, lens))
    assert np.array_equal(t.cpu().numpy(), want)
    assert np.array_equal(ts.cpu().numpy(), want_st)
    # host mode, out of place: bytes outside the streams keep the output buffer's contents
    hs = states.copy()
    out = np.full_like(data, 0xA5)
    brb.rc4_crypt_batch(hs, data, offs, lens, out=out)
    mask = np.zeros(data.size, bool)
    for o, n in zip(offs.tolist(), lens.tolist()):
        mask[o:o + n] = True
    assert np.array_equal(out[mask], want[mask]) and np.all(out[~mask] == 0xA5)
    assert np.array_equal(hs, want_st)


@pytest.mark.gpu
def test_rc4_state_carries_across_calls(brb, orc, torch_dev, rc4_pair):
    n = 200
    states = brb.rc4_states(_keys(n, 5))
    ts = _to(torch_dev, states)
    ost = states.copy()
    for call in range(4):
        lens = np.random.default_rng(call).integers(0, 300, n)
        offs, lens, total = _layout(lens, 7 + call, call)
        data = workload.gen_records(SEED + call, 0, 1, total + 4)
        ost, want = _oracle_crypt(orc, ost, data, offs, lens)
        t = _to(torch_dev, data)
        brb.rc4_crypt_batch(ts, t, _to(torch_dev, offs), _to(torch_dev, lens))
        assert np.array_equal(t.cpu().numpy(), want), call
    assert np.array_equal(ts.cpu().numpy(), ost)


@pytest.mark.gpu
def test_rc4_golden_streams(brb, torch_dev, golden, rc4_pair):
    for v in golden["rc4"]["streams"]:
        st = brb.rc4_states([bytes.fromhex(v["key"])])
        data = np.frombuffer(bytes.fromhex(v["data"]), np.uint8).copy()
        pos = 0
        for n, want in zip(v["lens"], v["out"]):
            seg = data[pos:pos + n].copy()
            brb.rc4_crypt_batch(st, seg, np.array([0], np.uint64), np.array([n], np.uint32))
            assert seg.tobytes().hex() == want
            pos += n
        assert st[0].tobytes().hex() == v["state_after"]


def _oracle_frames(orc, states, payload, offs, lens, salts, frames, foffs):
    st = states.copy()
    fr = frames.copy()
    for i in range(len(offs)):
        o, n, fo = int(offs[i]), int(lens[i]), int(foffs[i])
        s2, f = orc.rc4md5_frame(st[i].tobytes(), payload[o:o + n].tobytes(), int(salts[i]))
        st[i] = np.frombuffer(s2, np.uint8)
        fr[fo:fo + 30 + n] = np.frombuffer(f, np.uint8)
    return st, fr


@pytest.fixture(params=[1, 0], ids=["pair", "single"])
def rc4md5_pair(request, brb):
    """Test option rc4md5_pair: 1 the keystream + partner wave-pair frame / open kernels (default), 0
    one wave per connection."""
    with brb.TestOption("rc4md5_pair", request.param):
        yield request.param


@pytest.mark.gpu
@pytest.mark.parametrize("fbase", [0, 1, 2, 3])
def test_rc4md5_frame_batch(brb, orc, torch_dev, fbase, rc4md5_pair):
    lens = (RAGGED * 4)[: 100]
    offs, lens, total = _layout(lens, 3, 1)
    payload = workload.gen_records(SEED, 7, 1, total + 4)
    foffs, _, ftotal = _layout([30 + int(x) for x in lens], 9, fbase)
    salts = np.array([(0x9E3779B9 * (i + 1)) & 0xFFFFFFFF for i in range(len(offs))], np.uint64)
    states = brb.rc4_states(_keys(len(offs), 8))
    frames0 = np.full(ftotal + 8, 0x5A, np.uint8)
    want_st, want = _oracle_frames(orc, states, payload, offs, lens, salts, frames0, foffs)
    # device mode
    ts, tf = _to(torch_dev, states), _to(torch_dev, frames0)
    brb.rc4md5_frame_batch(ts, _to(torch_dev, payload), _to(torch_dev, offs), _to(torch_dev, lens),
                           _to(torch_dev, salts), tf, _to(torch_dev, foffs))
    assert np.array_equal(tf.cpu().numpy(), want)
    assert np.array_equal(ts.cpu().numpy(), want_st)
    # host mode
    hs, hf = states.copy(), frames0.copy()
    brb.rc4md5_frame_batch(hs, payload, offs, lens, salts, hf, foffs)
    assert np.array_equal(hf, want) and np.array_equal(hs, want_st)


@pytest.mark.gpu
def test_rc4md5_golden_frames(brb, golden):
    for v in golden["rc4"]["frames"]:
        payload = np.frombuffer(bytes.fromhex(v["payload"]) + b"\0", np.uint8).copy()
        n = len(payload) - 1
        st = brb.rc4_states([bytes.fromhex(v["key"])])
        fr = np.zeros(30 + n, np.uint8)
        brb.rc4md5_frame_batch(st, payload, np.array([0], np.uint64), np.array([n], np.uint32),
                               np.array([v["salt"]], np.uint64), fr, np.array([0], np.uint64))
        assert fr.tobytes().hex() == v["frame"] and st[0].tobytes().hex() == v["state_after"]


@pytest.mark.gpu
@pytest.mark.parametrize("base", [0, 1, 2, 3])
def test_rc4md5_open_batch(brb, orc, torch_dev, base, rc4md5_pair):
    """Frames written by the oracle are opened on the GPU; corrupted / short frames are rejected."""
    lens = (RAGGED * 4)[: 108]
    keys = _keys(len(lens), 12)
    rng = np.random.default_rng(base)
    frames, flens, expect_valid = [], [], []
    for i, n in enumerate(lens):
        payload = workload.gen_records(SEED, 100 + i, 1, n).tobytes() if n else b""
        _, fr = orc.rc4md5_frame(orc.rc4_init(keys[i]), payload, i)
        fr = bytearray(fr)
        kind = i % 6
        if kind == 3:                    # corrupt the tag, the digest or the payload
            pos = int(rng.choice([8, 10, 12, 13, 20, 28] + ([30, len(fr) - 1] if n else [])))
            fr[pos] ^= 0x40
        elif kind == 5 and n < 40:       # truncated below the header
            fr = fr[: int(rng.integers(0, 30))]
        frames.append(bytes(fr))
        flens.append(len(fr))
    offs, flens, total = _layout(flens, 4, base)
    buf = np.zeros(total + 8, np.uint8)
    for o, f in zip(offs.tolist(), frames):
        buf[o:o + len(f)] = np.frombuffer(f, np.uint8)
    states = brb.rc4_states(keys)
    want_buf, want_st, want_ok = buf.copy(), states.copy(), []
    for i, (o, f) in enumerate(zip(offs.tolist(), frames)):
        s2, dec, ok = orc.rc4md5_open(states[i].tobytes(), f)
        want_st[i] = np.frombuffer(s2, np.uint8)
        want_buf[o:o + len(f)] = np.frombuffer(dec, np.uint8)
        want_ok.append(ok)
    want_ok = np.array(want_ok, np.uint8)
    assert 0 < want_ok.sum() < len(want_ok)
    # device mode, in place
    ts, tb = _to(torch_dev, states), _to(torch_dev, buf)
    _, valid = brb.rc4md5_open_batch(ts, tb, _to(torch_dev, offs), _to(torch_dev, flens))
    assert np.array_equal(tb.cpu().numpy(), want_buf)
    assert np.array_equal(ts.cpu().numpy(), want_st)
    assert np.array_equal(valid.cpu().numpy(), want_ok)
    # host mode, out of place
    hs, out = states.copy(), np.zeros_like(buf)
    _, hv = brb.rc4md5_open_batch(hs, buf, offs, flens, out=out)
    assert np.array_equal(hv, want_ok) and np.array_equal(hs, want_st)
    for o, n in zip(offs.tolist(), flens.tolist()):
        assert np.array_equal(out[o:o + n], want_buf[o:o + n])


@pytest.mark.gpu
def test_rc4md5_round_trip_large(brb, torch_dev, rc4md5_pair):
    """Frame on the GPU, open on the GPU: 4096 connections x 1500 B plus a few 64 KiB payloads."""
    torch = torch_dev
    lens = [1500] * 4096 + [65536, 65535, 65537]
    n = len(lens)
    offs, lens, total = _layout(lens)
    payload = workload.gen_records(SEED, 0, 1, total)
    foffs, flens, ftotal = _layout([30 + int(x) for x in lens])
    keys = _keys(n, 21)
    wst, rst = _to(torch, brb.rc4_states(keys)), _to(torch, brb.rc4_states(keys))
    frames = torch.zeros(ftotal, dtype=torch.uint8, device="cuda")
    salts = _to(torch, np.arange(n, dtype=np.uint64))
    brb.rc4md5_frame_batch(wst, _to(torch, payload), _to(torch, offs), _to(torch, lens), salts, frames,
                           _to(torch, foffs))
    _, valid = brb.rc4md5_open_batch(rst, frames, _to(torch, foffs), _to(torch, flens))
    assert int(valid.sum()) == n
    assert torch.equal(wst, rst)          # both ends consumed the same keystream
    fr = frames.cpu().numpy()
    for i in (0, 1, 4095, n - 1):
        o, fo, m = int(offs[i]), int(foffs[i]), int(lens[i])
        assert fr[fo + 30:fo + 30 + m].tobytes() == payload[o:o + m].tobytes()
        assert fr[fo + 13:fo + 29].tobytes() == hashlib.md5(payload[o:o + m].tobytes()).digest()


@pytest.mark.gpu
def test_rc4_crypt_full_shape(brb, orc, torch_dev):
    """The f1 bench shape at full size: 65 536 connections x 1500 B through BRB_RC4_CryptBatch (device
    mode, in place), every stream's output and final state against the oracle's BRB_RC4_Crypt."""
    torch = torch_dev
    n, L = 65536, 1500
    data = workload.gen_records(SEED + 2, 0, n, L)
    rng = np.random.default_rng(65536)
    keys = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(n)]
    states = brb.rc4_states(keys)
    offs = np.arange(n, dtype=np.uint64) * L
    lens = np.full(n, L, np.uint32)
    ts, td = _to(torch, states), _to(torch, data)
    brb.rc4_crypt_batch(ts, td, _to(torch, offs), _to(torch, lens))
    got, got_st = td.cpu().numpy(), ts.cpu().numpy()
    for i in range(n):
        s2, ob = orc.rc4_crypt(states[i].tobytes(), data[i * L:(i + 1) * L].tobytes())
        assert got[i * L:(i + 1) * L].tobytes() == ob, i
        assert got_st[i].tobytes() == s2, i


@pytest.mark.gpu
def test_rc4md5_full_shape(brb, orc, torch_dev):
    """The rc4md5 bench shape at full size: 65 536 connections x 1500-byte payloads framed on the GPU
    (BRB_RC4MD5_FrameBatch) equal the oracle's frames and write states byte for byte; opened on the
    GPU (BRB_RC4MD5_OpenBatch) every frame validates, decrypts to its payload, and the read states
    equal the oracle's open of the same frames."""
    torch = torch_dev
    n, L = 65536, 1500
    payload = workload.gen_records(SEED + 3, 0, n, L)
    rng = np.random.default_rng(65537)
    keys = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(n)]
    st0 = brb.rc4_states(keys)
    offs = np.arange(n, dtype=np.uint64) * L
    lens = np.full(n, L, np.uint32)
    F = L + 30
    foffs = np.arange(n, dtype=np.uint64) * F
    flens = np.full(n, F, np.uint32)
    salts = rng.integers(0, 2**32, n, dtype=np.uint64)
    want_st, want_fr = st0.copy(), np.zeros(n * F, np.uint8)
    orc.rc4md5_frame_batch(want_st, payload, offs, lens, salts, want_fr, foffs, threads=16)
    ws, fr = _to(torch, st0), torch.zeros(n * F, dtype=torch.uint8, device="cuda")
    brb.rc4md5_frame_batch(ws, _to(torch, payload), _to(torch, offs), _to(torch, lens), _to(torch, salts), fr,
                           _to(torch, foffs))
    assert np.array_equal(fr.cpu().numpy(), want_fr)
    assert np.array_equal(ws.cpu().numpy(), want_st)
    want_rs, want_ok = st0.copy(), np.zeros(n, np.uint8)
    want_pt = want_fr.copy()
    orc.rc4md5_open_batch(want_rs, want_pt, foffs, flens, want_ok, threads=16)
    rs = _to(torch, st0)
    _, valid = brb.rc4md5_open_batch(rs, fr, _to(torch, foffs), _to(torch, flens))
    assert int(valid.sum()) == n and want_ok.all()
    assert np.array_equal(rs.cpu().numpy(), want_rs)
    got = fr.cpu().numpy().reshape(n, F)
    assert np.array_equal(got, want_pt.reshape(n, F))
    assert np.array_equal(got[:, 30:], payload.reshape(n, L))


@pytest.mark.gpu
@pytest.mark.parametrize("sector", [1, 0])
def test_rc4_sector_sink_ragged(brb, orc, sector):
    """Both output sinks of the RC4 pass on ragged, packed streams at every byte offset, device mode
    in place, against the oracle: brb_io::SectorSnk (whole aligned sectors, the default for every
    output) and the per-stream Snk it replaced (kept for A/B runs), forced with the "rc4_sector"
    test option (BRB_CryptoGPU_TestOption)."""
    import torch
    rng = np.random.default_rng(11)
    with brb.TestOption("rc4_sector", sector):
        for base in (0, 1, 2, 3):
            lens = rng.integers(0, 3000, 257).astype(np.uint32)
            gaps = rng.integers(0, 6, 257)
            offs = (base + np.concatenate([[0], np.cumsum(lens[:-1].astype(np.int64) + gaps[:-1])])).astype(np.uint64)
            total = int(offs[-1] + lens[-1]) + 8
            data = workload.gen_records(0x5EED00A1, base, 1, total)
            keys = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(len(offs))]
            states = brb.rc4_states(keys)
            want = data.copy()
            for i, (o, n) in enumerate(zip(offs.tolist(), lens.tolist())):
                s2, ob = orc.rc4_crypt(states[i].tobytes(), data[o:o + n].tobytes())
                want[o:o + n] = np.frombuffer(ob, np.uint8)
            t = torch.from_numpy(data).cuda()
            brb.rc4_crypt_batch(torch.from_numpy(states).cuda(), t, torch.from_numpy(offs).cuda(),
                                torch.from_numpy(lens).cuda())
            assert np.array_equal(t.cpu().numpy(), want), base


@pytest.mark.gpu
def test_rc4_ragged_out_of_place(brb, orc, rc4_pair):
    """Ragged, packed streams (0..3000 B, the block-edge lengths first) at every input byte offset,
    in place and out of place into an output buffer shifted so that output and input alignments
    differ; device mode, against the oracle, states included; bytes between streams untouched."""
    import torch
    rng = np.random.default_rng(11)
    for base in (0, 1, 2, 3):
        for shift in (None, 0, 1, 5, 37, 63):
            lens = rng.integers(0, 3000, 257).astype(np.uint32)
            lens[:8] = [0, 1, 63, 64, 65, 127, 128, 129]
            gaps = rng.integers(0, 6, 257)
            offs = (base + np.concatenate([[0], np.cumsum(lens[:-1].astype(np.int64) + gaps[:-1])])).astype(np.uint64)
            total = int(offs[-1] + lens[-1]) + 8
            data = workload.gen_records(0x5EED00A1, base, 1, total)
            keys = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(len(offs))]
            states = brb.rc4_states(keys)
            want = data.copy()
            want_st = states.copy()
            for i, (o, n) in enumerate(zip(offs.tolist(), lens.tolist())):
                s2, ob = orc.rc4_crypt(states[i].tobytes(), data[o:o + n].tobytes())
                want[o:o + n] = np.frombuffer(ob, np.uint8)
                want_st[i] = np.frombuffer(s2, np.uint8)
            t = torch.from_numpy(data).cuda()
            st = torch.from_numpy(states).cuda()
            if shift is None:
                brb.rc4_crypt_batch(st, t, torch.from_numpy(offs).cuda(), torch.from_numpy(lens).cuda())
                got = t.cpu().numpy()
            else:
                fill = np.full(total + 64, 0xA5, np.uint8)
                big = torch.from_numpy(fill).cuda()
                out = big[shift:shift + total]
                brb.rc4_crypt_batch(st, t, torch.from_numpy(offs).cuda(), torch.from_numpy(lens).cuda(), out=out)
                got = out.cpu().numpy()
                # bytes outside the streams stay untouched
                want = np.where(_covered(offs, lens, total), want, np.uint8(0xA5))
                assert np.array_equal(big.cpu().numpy()[:shift], fill[:shift])
            assert np.array_equal(got, want), (base, shift)
            assert np.array_equal(st.cpu().numpy(), want_st), (base, shift)


def _covered(offs, lens, total):
    m = np.zeros(total, bool)
    for o, n in zip(offs.tolist(), lens.tolist()):
        m[o:o + n] = True
    return m


@pytest.mark.gpu
def test_streams_beyond_4gib(brb, orc, torch_dev):
    """Stream and record offsets past 2^32 in one 4.5 GiB device buffer: 600 streams (0..3000 bytes,
    some straddling byte offsets 2^31 and 2^32, some ending at the buffer's last byte) through the
    variable-length MD5 batch and the RC4 pass (in place), against hashlib and the oracle on host
    copies of just those streams; states included."""
    torch = torch_dev
    total = 9 << 29
    words = torch.empty(total // 8, dtype=torch.int64, device="cuda")
    g = torch.Generator(device="cuda")
    g.manual_seed(0x4B1C)
    words.random_(generator=g)
    d = words.view(torch.uint8)
    rng = np.random.default_rng(11)
    n = 600
    lens = rng.integers(0, 3001, n).astype(np.uint32)
    offs = rng.integers(0, total - 3001, n).astype(np.uint64)
    for i, o in enumerate([(1 << 31) - 700, (1 << 32) - 700, (1 << 32) - 1, 1 << 32, (1 << 32) + 3]):
        offs[i], lens[i] = o, 1500
    offs[5], lens[5] = total - 1500, 1500
    offs[6], lens[6] = total - 7, 7
    # non-overlapping streams (the RC4 pass writes in place): drop any that overlaps an earlier one
    order = np.argsort(offs, kind="stable")
    keep, end = [], 0
    for i in order.tolist():
        if int(offs[i]) >= end:
            keep.append(i)
            end = int(offs[i]) + int(lens[i])
    keep = np.array(sorted(keep))
    offs, lens = offs[keep], lens[keep]
    host = [d[int(o):int(o) + int(m)].cpu().numpy() for o, m in zip(offs, lens)]
    to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()   # noqa: E731
    dig = brb.md5_batch(d, to(offs.view(np.int64)), to(lens.view(np.int32))).cpu().numpy()
    for i, h in enumerate(host):
        assert dig[i].tobytes() == hashlib.md5(h.tobytes()).digest(), f"md5 stream {i} at {int(offs[i])}"
    states = brb.rc4_states(_keys(len(offs), 9))
    ts = to(states)
    brb.rc4_crypt_batch(ts, d, to(offs.view(np.int64)), to(lens.view(np.int32)))
    got_st = ts.cpu().numpy()
    for i, h in enumerate(host):
        s2, ob = orc.rc4_crypt(states[i].tobytes(), h.tobytes())
        o, m = int(offs[i]), int(lens[i])
        assert d[o:o + m].cpu().numpy().tobytes() == ob, f"rc4 stream {i} at {o}"
        assert got_st[i].tobytes() == s2, f"rc4 state {i}"
    del words, d
    torch.cuda.empty_cache()


@pytest.mark.gpu
def test_frames_beyond_4gib(brb, orc, torch_dev):
    """The RC4+MD5 frame and open kernels with payloads read from, and frames written to, byte
    offsets past 2^31 and 2^32 of one 4.5 GiB device buffer: 300 connections (0..3000-byte
    payloads), every frame against the oracle's frame, then opened in place (valid, payload back,
    both ends' states equal)."""
    torch = torch_dev
    total = 9 << 29
    words = torch.empty(total // 8, dtype=torch.int64, device="cuda")
    g = torch.Generator(device="cuda")
    g.manual_seed(0x4B1F)
    words.random_(generator=g)
    d = words.view(torch.uint8)
    rng = np.random.default_rng(41)
    n = 300
    lens = rng.integers(0, 3001, n).astype(np.uint32)
    # payloads in the lower 4 GiB + 256 MiB (some straddling 2^31 / 2^32), frames back to back
    # (3-byte gaps, odd start) above them, all past 2^32 + 256 MiB
    offs = rng.integers(0, (1 << 32) + (256 << 20), n).astype(np.uint64)
    offs[0], offs[1], lens[0], lens[1] = (1 << 31) - 900, (1 << 32) - 900, 2000, 2000
    foffs = np.zeros(n, np.uint64)
    foffs[1:] = np.cumsum(lens.astype(np.uint64) + 30 + 3)[:-1]
    foffs += (1 << 32) + (256 << 20) + 8191
    # every range inside the buffer (checked on the host before any kernel runs)
    assert int((offs + lens).max()) <= (1 << 32) + (256 << 20) + 3000 < int(foffs[0])
    assert int(foffs[-1]) + 30 + int(lens[-1]) <= total
    payload = [d[int(o):int(o) + int(m)].cpu().numpy().tobytes() for o, m in zip(offs, lens)]
    salts = np.array([(0x9E3779B9 * (i + 3)) & 0xFFFFFFFF for i in range(n)], np.uint64)
    keys = _keys(n, 41)
    states = brb.rc4_states(keys)
    to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()   # noqa: E731
    ws, rs = to(states), to(states)
    brb.rc4md5_frame_batch(ws, d, to(offs.view(np.int64)), to(lens.view(np.int32)), to(salts.view(np.int64)), d,
                           to(foffs.view(np.int64)))
    want_st = []
    for i in range(n):
        s2, f = orc.rc4md5_frame(states[i].tobytes(), payload[i], int(salts[i]))
        fo = int(foffs[i])
        assert d[fo:fo + 30 + int(lens[i])].cpu().numpy().tobytes() == f, f"frame {i} at {fo}"
        want_st.append(s2)
    assert ws.cpu().numpy().tobytes() == b"".join(want_st)
    flens = (lens + 30).astype(np.uint32)
    _, valid = brb.rc4md5_open_batch(rs, d, to(foffs.view(np.int64)), to(flens.view(np.int32)))
    assert bool(valid.cpu().numpy().astype(bool).all())
    assert torch.equal(ws, rs)
    for i in range(n):
        fo = int(foffs[i])
        assert d[fo + 30:fo + 30 + int(lens[i])].cpu().numpy().tobytes() == payload[i], f"opened {i}"
    del words, d
    torch.cuda.empty_cache()


@pytest.mark.gpu
def test_rc4_pair_fault_reported(brb, orc, torch_dev):
    """A protocol fault in the keystream + I/O wave pair (test option pair_stall: the first I/O wave
    never hands a block over, so both waves' bounded waits give up) is reported as BRB_BATCH_FAULT
    (-4, pair_fault.h) in host and device mode, never returned as a result; the next call on the
    same thread is clean and exact."""
    torch = torch_dev
    n = 128
    offs, lens, total = _layout([4096] * n)
    data = workload.gen_records(SEED + 9, 0, 1, total)
    states = brb.rc4_states(_keys(n, 33))
    with brb.TestOption("rc4_pair", 1), brb.TestOption("pair_stall", 1):
        with pytest.raises(RuntimeError, match=r"returned -4: wave-pair protocol fault"):
            brb.rc4_crypt_batch(states.copy(), data.copy(), offs, lens)
        with pytest.raises(RuntimeError, match=r"returned -4: wave-pair protocol fault"):
            brb.rc4_crypt_batch(_to(torch, states), _to(torch, data), _to(torch, offs), _to(torch, lens))
    st, out = states.copy(), data.copy()
    brb.rc4_crypt_batch(st, out, offs, lens)
    want_st, want = _oracle_crypt(orc, states, data, offs, lens)
    assert np.array_equal(out, want) and np.array_equal(st, want_st)


@pytest.mark.gpu
def test_rc4md5_pair_fault_reported(brb, orc, torch_dev):
    """A protocol fault in the RC4+MD5 frame / open wave pairs (test option pair_stall: the first
    partner wave stages its blocks but never hands one over) is reported as BRB_BATCH_FAULT (-4) by
    FrameBatch and OpenBatch in host and device mode; the next calls on the thread are exact."""
    torch = torch_dev
    n = 128
    offs, lens, total = _layout([1500] * (n - 2) + [0, 200])
    payload = workload.gen_records(SEED + 10, 0, 1, total + 4)
    foffs, _, ftotal = _layout([30 + int(x) for x in lens])
    salts = np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15 & 0xFFFFFFFF)
    states = brb.rc4_states(_keys(n, 41))
    frames0 = np.zeros(ftotal + 8, np.uint8)
    want_st, want_fr = _oracle_frames(orc, states, payload, offs, lens, salts, frames0, foffs)
    flens = (lens + 30).astype(np.uint32)
    with brb.TestOption("rc4md5_pair", 1), brb.TestOption("pair_stall", 1):
        with pytest.raises(RuntimeError, match=r"returned -4: wave-pair protocol fault"):
            brb.rc4md5_frame_batch(states.copy(), payload, offs, lens, salts, frames0.copy(), foffs)
        with pytest.raises(RuntimeError, match=r"returned -4: wave-pair protocol fault"):
            brb.rc4md5_frame_batch(_to(torch, states), _to(torch, payload), _to(torch, offs), _to(torch, lens),
                                   _to(torch, salts), _to(torch, frames0), _to(torch, foffs))
        with pytest.raises(RuntimeError, match=r"returned -4: wave-pair protocol fault"):
            brb.rc4md5_open_batch(states.copy(), want_fr.copy(), foffs, flens)
        with pytest.raises(RuntimeError, match=r"returned -4: wave-pair protocol fault"):
            brb.rc4md5_open_batch(_to(torch, states), _to(torch, want_fr), _to(torch, foffs), _to(torch, flens))
    hs, hf = states.copy(), frames0.copy()
    brb.rc4md5_frame_batch(hs, payload, offs, lens, salts, hf, foffs)
    assert np.array_equal(hf, want_fr) and np.array_equal(hs, want_st)
    os_, buf = states.copy(), want_fr.copy()
    _, valid = brb.rc4md5_open_batch(os_, buf, foffs, flens)
    assert valid.tolist() == [1] * n and np.array_equal(os_, want_st)
    for i in range(n):
        o, m = int(foffs[i]), int(lens[i])
        assert buf[o + 30:o + 30 + m].tobytes() == payload[int(offs[i]):int(offs[i]) + m].tobytes(), i


@pytest.mark.gpu
def test_async_pair_fault_check(brb, orc, torch_dev):
    """Device-mode BRB_BATCH_ASYNC calls return before their kernels run, so a wave-pair fault
    (pair_stall) cannot be their return code: BRB_CryptoGPU_AsyncFaultCheck() reports it once the
    caller has synchronised (-4, then cleared), and stays clean after a clean async call."""
    torch = torch_dev
    n = 128
    offs, lens, total = _layout([4096] * n)
    data = workload.gen_records(SEED + 11, 0, 1, total)
    states = brb.rc4_states(_keys(n, 43))
    brb.async_fault_check()                                  # nothing pending on this thread
    args = (_to(torch, offs), _to(torch, lens))
    with brb.TestOption("rc4_pair", 1), brb.TestOption("pair_stall", 1):
        brb.rc4_crypt_batch(_to(torch, states), _to(torch, data), *args, async_=True)
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match=r"AsyncFaultCheck returned -4: wave-pair protocol fault"):
        brb.async_fault_check()
    brb.async_fault_check()                                  # the report was cleared
    ts, td = _to(torch, states), _to(torch, data)
    with brb.TestOption("rc4_pair", 1):
        brb.rc4_crypt_batch(ts, td, *args, async_=True)
    torch.cuda.synchronize()
    brb.async_fault_check()
    want_st, want = _oracle_crypt(orc, states, data, offs, lens)
    assert np.array_equal(td.cpu().numpy(), want) and np.array_equal(ts.cpu().numpy(), want_st)


@pytest.mark.gpu
def test_async_fault_words_are_per_thread(brb, orc, torch_dev):
    """The async fault report is the calling thread's: a stalled async call on one thread is seen by
    that thread's check only; another thread's async calls and checks stay clean."""
    import threading
    torch = torch_dev
    n = 128
    offs, lens, total = _layout([2048] * n)
    data = workload.gen_records(SEED + 12, 0, 1, total)
    states = brb.rc4_states(_keys(n, 44))
    res = {}

    def clean():
        ts, td = _to(torch, states), _to(torch, data)
        for _ in range(3):
            brb.rc4_crypt_batch(ts, td, _to(torch, offs), _to(torch, lens), async_=True)
        torch.cuda.synchronize()
        try:
            brb.async_fault_check()
            res["clean"] = "ok"
        except RuntimeError as e:
            res["clean"] = str(e)

    with brb.TestOption("rc4_pair", 1), brb.TestOption("pair_stall", 1):
        brb.rc4_crypt_batch(_to(torch, states), _to(torch, data), _to(torch, offs), _to(torch, lens), async_=True)
    torch.cuda.synchronize()
    th = threading.Thread(target=clean)
    th.start()
    th.join()
    assert res["clean"] == "ok"
    with pytest.raises(RuntimeError, match="returned -4"):
        brb.async_fault_check()


@pytest.mark.gpu
def test_thread_cleanup_drains_async_pair_calls(brb, orc, torch_dev):
    """a device-mode async call of a wave-pair kernel returns before the kernel runs, and
    the kernel writes the calling thread's fault word.  A thread that cleans up (ThreadCleanup, or
    its exit) with such a call still queued -- here behind ~0.1 s of spinning on the same stream --
    must not free the word under the kernel: cleanup drains the devices the thread armed the word
    on first.  The kernel's results are then the oracle's, and later calls on a fresh thread work."""
    import threading
    import time
    torch = torch_dev
    n = 128
    offs, lens, total = _layout([4096] * n)
    data = workload.gen_records(SEED + 13, 0, 1, total)
    states = brb.rc4_states(_keys(n, 45))
    ts, td = _to(torch, states), _to(torch, data)
    to, tl = _to(torch, offs), _to(torch, lens)
    torch.cuda.synchronize()
    res = {}

    def worker():
        s = torch.cuda.current_stream()
        torch.cuda._sleep(200_000_000)                     # the pair kernel queues behind this
        with brb.TestOption("rc4_pair", 1):
            brb.rc4_crypt_batch(ts, td, to, tl, stream=s, async_=True)
        t0 = time.perf_counter()
        brb.lib().BRB_CryptoGPU_ThreadCleanup()           # frees the async fault word: after the drain
        res["cleanup_s"] = time.perf_counter() - t0
        res["done"] = bool(torch.cuda.current_stream().query())

    th = threading.Thread(target=worker)
    th.start()
    th.join()
    assert res["done"], "ThreadCleanup returned with the thread's async pair kernel still queued"
    torch.cuda.synchronize()
    want_st, want = _oracle_crypt(orc, states, data, offs, lens)
    assert np.array_equal(td.cpu().numpy(), want) and np.array_equal(ts.cpu().numpy(), want_st)
    brb.async_fault_check()
