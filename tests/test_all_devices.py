"""The multi-device paths (advisor r02) against the oracle.

* BRB_BATCH_ALL_DEVICES on the multi-range batch calls (RC4, frame, open, base64, segment digests;
  MetaData has its own test in test_metadata.py) and on the fixed / variable digests and Blowfish: the records split into contiguous
  ranges, one per part, run concurrently from per-part worker threads.
* BRB_BATCHER_ALL_DEVICES: connection c lives on part c % G (as its connection c // G) with both
  RC4 states; one Flush enqueues every part's round before waiting for any.

A one-GPU box would only ever take the one-part shortcut, so the "devices" test option
(BRB_CryptoGPU_TestOption) forces G parts mapped onto the visible devices (part g on device
g % count): the worker threads, per-part results and callbacks of the concurrent path all run.  The
8-GPU placement itself is unmeasured here."""
import numpy as np
import pytest

from brb_framework_amd import workload


def test_connection_partition_model():
    """CPU: the partition rule both the all-devices batcher and the tests below assume is a
    bijection of [0, max_conns) onto the parts' local connection ids (each part sized by
    ceil((max_conns - g) / G), transform_batcher.hip Create)."""
    for max_conns in (1, 2, 7, 64, 300, 1001):
        for G in (1, 2, 3, 8):
            seen = set()
            sizes = [(max_conns - g + G - 1) // G for g in range(G)]
            for c in range(max_conns):
                g, local = workload.conn_part(c, G)
                assert 0 <= g < G and 0 <= local < sizes[g]
                seen.add((g, local))
            assert len(seen) == max_conns == sum(sizes)


def test_record_split_model():
    """CPU: contiguous ranges [g n / G, (g + 1) n / G) cover every record once (workload.shard,
    the rule split_devices applies)."""
    for n in (0, 1, 5, 64, 1000, 65537):
        for G in (1, 2, 3, 8):
            cover = []
            for g in range(G):
                lo, hi = workload.shard(n, g, G)
                cover.extend(range(lo, hi))
            assert cover == list(range(n))


@pytest.fixture(scope="module")
def torch_dev(brb):
    import torch
    assert torch.cuda.is_available(), "no HIP device visible to torch"
    assert brb.gpu_available(), brb.lib().BRB_CryptoGPU_LastError()
    return torch


def _layout(lens, gap, seed):
    rng = np.random.default_rng(seed)
    offs, pos = [], 3
    for L in lens:
        offs.append(pos)
        pos += int(L) + int(rng.integers(0, gap + 1))
    return np.array(offs, np.uint64), np.array(lens, np.uint32), pos + 8


def _keys(n, salt=0):
    return [bytes([(i * 7 + salt) & 255, (i >> 8) & 255, 3, 5, salt & 255]) for i in range(n)]


@pytest.mark.gpu
@pytest.mark.parametrize("parts", [3, 1])
@pytest.mark.parametrize("order", ["submission", "reversed"])
def test_rc4_frame_open_all_devices(brb, orc, torch_dev, parts, order):
    """RC4 pass, frame and open in host mode with BRB_BATCH_ALL_DEVICES: states go with their streams.
    "reversed": the streams' byte ranges run backwards through the buffer, so the parts' spans
    interleave and the call must take the one-device path -- same results."""
    rng = np.random.default_rng(parts)
    n = 301
    lens = rng.integers(0, 3000, n)
    lens[:5] = [0, 1, 63, 64, 65]
    if order == "reversed":           # stream i at the place the forward layout gives stream n-1-i
        fwd, _, total = _layout(lens[::-1], 5, 1)
        offs, lens = np.ascontiguousarray(fwd[::-1]), np.ascontiguousarray(lens, np.uint32)
    else:
        offs, lens, total = _layout(lens, 5, 1)
    data = workload.gen_records(0x5EED00C1, parts, 1, total)
    states = brb.rc4_states(_keys(n))
    want, want_st = data.copy(), states.copy()
    for i, (o, L) in enumerate(zip(offs.tolist(), lens.tolist())):
        s2, ob = orc.rc4_crypt(states[i].tobytes(), data[o:o + L].tobytes())
        want[o:o + L] = np.frombuffer(ob, np.uint8)
        want_st[i] = np.frombuffer(s2, np.uint8)
    with brb.TestOption("devices", parts):
        hs, hd = states.copy(), data.copy()
        brb.rc4_crypt_batch(hs, hd, offs, lens, all_devices=True)
        assert np.array_equal(hd, want) and np.array_equal(hs, want_st)
        # frames of the same payloads (write side), then open them (read side)
        foffs, _, ftotal = _layout([30 + int(x) for x in lens], 3, 2)
        salts = np.arange(n, dtype=np.uint64) * 977
        ws = brb.rc4_states(_keys(n, 9))
        frames = np.full(ftotal, 0x5A, np.uint8)
        wframes, wws = frames.copy(), ws.copy()
        for i, (o, L) in enumerate(zip(offs.tolist(), lens.tolist())):
            s2, fr = orc.rc4md5_frame(ws[i].tobytes(), data[o:o + L].tobytes(), int(salts[i]))
            wws[i] = np.frombuffer(s2, np.uint8)
            wframes[int(foffs[i]):int(foffs[i]) + 30 + L] = np.frombuffer(fr, np.uint8)
        hws, hf = ws.copy(), frames.copy()
        brb.rc4md5_frame_batch(hws, data, offs, lens, salts, hf, foffs, all_devices=True)
        assert np.array_equal(hf, wframes) and np.array_equal(hws, wws)
        rs = brb.rc4_states(_keys(n, 9))
        flens = lens + 30
        hrs, hb = rs.copy(), hf.copy()
        _, valid = brb.rc4md5_open_batch(hrs, hb, foffs, flens, all_devices=True)
        assert valid.all() and np.array_equal(hrs, wws)
        for i, (o, L) in enumerate(zip(offs.tolist(), lens.tolist())):
            assert hb[int(foffs[i]) + 30:int(foffs[i]) + 30 + L].tobytes() == data[o:o + L].tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("parts", [4, 1])
def test_base64_segments_all_devices(brb, orc, torch_dev, parts):
    rng = np.random.default_rng(40 + parts)
    n = 257
    lens = rng.integers(0, 2500, n)
    offs, lens, total = _layout(lens, 3, 4)
    data = workload.gen_records(0x5EED00C2, parts, 1, total)
    want = [orc.b64_encode(data[int(o):int(o) + int(L)].tobytes()) for o, L in zip(offs, lens)]
    elens = np.array([len(w) for w in want], np.uint32)
    eoffs = np.zeros(n, np.uint64)
    eoffs[1:] = np.cumsum(elens.astype(np.uint64) + 1)[:-1]
    with brb.TestOption("devices", parts):
        out = np.full(int(eoffs[-1] + elens[-1] + 8), 0xEE, np.uint8)
        brb.base64_encode_batch(data, offs, lens, out, eoffs, all_devices=True)
        for i in range(n):
            assert out[int(eoffs[i]):int(eoffs[i]) + int(elens[i])].tobytes() == want[i]
            assert out[int(eoffs[i]) + int(elens[i])] == 0xEE
        cap = 3 * (elens // 4)
        doffs = np.zeros(n, np.uint64)
        doffs[1:] = np.cumsum(cap.astype(np.uint64))[:-1]
        back = np.zeros(int(cap.sum()) + 8, np.uint8)
        got_len = brb.base64_decode_batch(out, eoffs, elens, back, doffs, all_devices=True)
        for i in range(n):
            w = orc.b64_decode(out[int(eoffs[i]):int(eoffs[i]) + int(elens[i])].tobytes())
            assert int(got_len[i]) == len(w) and back[int(doffs[i]):int(doffs[i]) + len(w)].tobytes() == w
        # segment digests: record i = its payload cut into up to three segments
        first = [0]
        soffs, slens = [], []
        for o, L in zip(offs.tolist(), lens.tolist()):
            cuts = sorted(rng.integers(0, L + 1, 2).tolist()) if L else [0, 0]
            for a, b in ((0, cuts[0]), (cuts[0], cuts[1]), (cuts[1], L)):
                soffs.append(o + a)
                slens.append(b - a)
            first.append(len(soffs))
        dg = brb.md5_batch_segments(data, np.array(soffs, np.uint64), np.array(slens, np.uint32),
                                    np.array(first, np.uint64), all_devices=True)
        assert np.array_equal(dg, orc.md5_batch(data, offs, lens, threads=8))


@pytest.mark.gpu
def test_line_forced_parts(brb, orc, torch_dev):
    """The line kernel under the host-mode split: three parts on their worker threads, launched
    concurrently (300 001 records: ~100 000 per part, 7 rounds of groups, partial last groups), twice."""
    L, n = 1500, 300_001
    data = workload.gen_records(0x5EED00C4, 0, n, L)
    want = orc.md5_batch_fixed(data, L, n, threads=8)
    with brb.TestOption("devices", 3):
        for _ in range(2):
            assert np.array_equal(brb.md5_batch_fixed(data, L, n, all_devices=True), want)


@pytest.mark.gpu
@pytest.mark.parametrize("parts", [3])
def test_digests_blowfish_forced_parts(brb, orc, torch_dev, parts):
    """The advisor's round-2 item: the concurrent split (worker threads, Pending, per-part results)
    of the fixed / variable digests and Blowfish, with G forced above the visible devices."""
    with brb.TestOption("devices", parts):
        L, n = 1500, 9001
        data = workload.gen_records(0x5EED00C3, 0, n, L)
        assert np.array_equal(brb.md5_batch_fixed(data, L, n, all_devices=True), orc.md5_batch_fixed(data, L, n, threads=8))
        assert np.array_equal(brb.sha1_batch_fixed(data, L, n, all_devices=True), orc.sha1_batch_fixed(data, L, n, threads=8))
        rng = np.random.default_rng(5)
        vl = rng.integers(0, 3000, 5000).astype(np.uint32)
        vo = rng.integers(0, data.size - 3000, 5000).astype(np.uint64)
        assert np.array_equal(brb.md5_batch(data, vo, vl, all_devices=True), orc.md5_batch(data, vo, vl, threads=8))
        nb = (1 << 20) + 3
        w = workload.gen_words(workload.SEEDS[4], 2 * nb)
        ctx = brb.blowfish_init(workload.CFG4_KEY)
        buf = w.copy()
        brb.blowfish_encrypt_batch(ctx, buf, all_devices=True)
        assert np.array_equal(buf, orc.bf_ecb(orc.bf_init(workload.CFG4_KEY), w.copy(), threads=8))
        brb.blowfish_decrypt_batch(ctx, buf, all_devices=True)
        assert np.array_equal(buf, w)


@pytest.mark.gpu
@pytest.mark.parametrize("pipelined", [False, True])
@pytest.mark.parametrize("zero_copy", [False, True])
@pytest.mark.parametrize("parts", [3, 1])
def test_batcher_all_devices(brb, orc, torch_dev, parts, zero_copy, pipelined):
    """BRB_BATCHER_ALL_DEVICES on a synthetic event loop (RC4+MD5): every connection's results come
    back in its own order and equal the per-buffer oracle, states included, with the connections
    spread over `parts` sub-batchers."""
    with brb.TestOption("devices", parts):
        C = 97
        rng = np.random.default_rng(parts * 10 + zero_copy * 2 + pipelined)
        keys = [rng.integers(0, 256, int(rng.integers(4, 32)), dtype=np.uint8).tobytes() for _ in range(C)]
        b = brb.TransformBatcher(C, 4 << 20, 2, zero_copy=zero_copy, pipelined=pipelined, all_devices=True)
        ours_r = [orc.rc4_init(k) for k in keys]
        ours_w = [orc.rc4_init(k) for k in keys]
        peer_w = [orc.rc4_init(k) for k in keys]
        for c in range(C):
            b.enable(c, keys[c])
        want = {c: [] for c in range(C)}
        got = {c: [] for c in range(C)}
        for rnd in range(5):
            for c in rng.permutation(C)[: int(rng.integers(C // 3, C))]:
                c = int(c)
                for _ in range(int(rng.integers(0, 3))):
                    n = int(rng.choice([0, 5, 64, 700, 1500]))
                    payload = workload.gen_records(0x5EED00C4 + rnd, c * 8, 1, n).tobytes() if n else b""
                    peer_w[c], frame = orc.rc4md5_frame(peer_w[c], payload, rnd * 1000 + c)
                    ours_r[c], dec, ok = orc.rc4md5_open(ours_r[c], frame)
                    want[c].append((0, dec, ok))
                    assert b.read(c, frame) == 1
                for _ in range(int(rng.integers(0, 2))):
                    n = int(rng.choice([0, 3, 1500]))
                    payload = workload.gen_records(0x5EED00C5 + rnd, c * 8, 1, n).tobytes() if n else b""
                    ours_w[c], frame = orc.rc4md5_frame(ours_w[c], payload, c + rnd)
                    want[c].append((1, frame, 1))
                    assert b.write(c, payload, c + rnd) == 1
            res = b.flush_async() if pipelined else b.flush()
            for conn, op, out, valid in res:
                got[conn].append((op, out, valid))
        for conn, op, out, valid in b.flush():
            got[conn].append((op, out, valid))
        for c in range(C):
            assert got[c] == want[c], c
            assert b.state(c, 0) == ours_r[c] and b.state(c, 1) == ours_w[c]
        b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("how", ["async", "sync"])
def test_batcher_all_devices_fault_poisons(brb, orc, torch_dev, how):
    """The round-6 poisoning contract (test_batcher.py::test_pipelined_fault_poisons_next_round)
    through BRB_BATCHER_ALL_DEVICES with the connections over 3 sub-batchers: round A faults (test
    option pair_stall) on every sub, round B was submitted behind it, and every sub poisons its own
    connections of A.  Compared per connection (subs deliver one after another)."""
    with brb.TestOption("devices", 3):
        rng = np.random.default_rng(77 if how == "async" else 78)
        C, CA = 96, 80
        keys = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(C)]
        b = brb.TransformBatcher(C, 4 << 20, 2, pipelined=True, all_devices=True)
        st = {}

        def rekey(conns):
            for c in conns:
                b.enable(c, keys[c])
                st[c] = [orc.rc4_init(keys[c]) for _ in range(3)]

        def submit(c, rnd):
            n = int(rng.choice([0, 17, 700, 1500]))
            payload = workload.gen_records(0x5EED00F9 + rnd, c, 1, n).tobytes() if n else b""
            r, w, pw = st[c]
            pw, frame = orc.rc4md5_frame(pw, payload, c)
            r, dec, ok = orc.rc4md5_open(r, frame)
            assert b.read(c, frame) == 1
            w, out = orc.rc4md5_frame(w, payload, rnd + c)
            assert b.write(c, payload, rnd + c) == 1
            st[c] = [r, w, pw]
            return [(0, dec, ok), (1, out, 1)]

        drop = [(0, b"", brb.TRANSFORM_DROPPED), (1, b"", brb.TRANSFORM_DROPPED)]
        want = {c: [] for c in range(C)}
        got = {c: [] for c in range(C)}

        def take(results):
            for conn, op, out, valid in results:
                got[conn].append((op, out, valid))

        rekey(range(C))
        for c in range(CA):
            submit(c, 0)
            want[c] += drop
        with brb.TestOption("rc4md5_pair", 1), brb.TestOption("pair_stall", 1):
            assert b.flush_async() == []
        for c in range(C):
            e = submit(c, 1)
            want[c] += drop if c < CA else e
        with pytest.raises(RuntimeError, match="dropped") as ei:
            b.flush_async() if how == "async" else b.flush()
        assert ei.value.code == brb.BATCH_DROPPED
        take(ei.value.results)
        assert b.read(0, b"refused") == -1 and b.write(CA - 1, b"refused", 0) == -1
        try:
            take(b.flush())
        except RuntimeError as e:                 # async: B's poisoned buffers come back here
            assert e.code == brb.BATCH_DROPPED
            take(e.results)
        for c in range(C):
            assert got[c] == want[c], c
        rekey(range(CA))
        for c in range(C):
            want[c] += submit(c, 3)
        take(b.flush())
        for c in range(C):
            assert got[c] == want[c], c
            assert b.state(c, 0) == st[c][0] and b.state(c, 1) == st[c][1]
        b.close()
