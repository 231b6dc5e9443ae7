"""Receive-loop batching: a synthetic event loop drives BRB_TransformBatcher.

Each round, a random subset of connections delivers 0..3 buffers (frames written by the peer with
the oracle's RC4+MD5 write side) and sends 0..2 buffers.  The batcher's results must equal what the
reference's per-buffer hook would produce for each connection in order (oracle), including the
RC4 states after every round, frame validity and tampered frames.  The kqueue loop itself
(ev_kq_base.c:589) is modelled, not run: libkqueue is not available here."""
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


def _check_round(got, expect, rnd):
    assert len(got) == len(expect), rnd
    for g, e in zip(got, expect):
        assert g[0] == e[0] and g[1] == e[1] and g[2] == e[2] and g[3] == e[3], (rnd, e[0], e[1])


@pytest.mark.parametrize("pipelined", [False, True])
@pytest.mark.parametrize("zero_copy", [False, True])
@pytest.mark.parametrize("algo", [1, 2])
def test_event_loop_rounds(brb, orc, torch_dev, algo, zero_copy, pipelined):
    """pipelined: BRB_BATCHER_PIPELINED, each round started with FlushAsync, whose results come
    back from the next round's FlushAsync (the last from Flush)."""
    _event_loop(brb, orc, algo, zero_copy, pipelined)


def test_event_loop_after_rc4_and_base64(brb, orc, torch_dev):
    """Regression, in the order that failed in round 2: a full-size RC4 pass and a
    base64 round trip enqueued on the default stream, then -- without waiting for them -- the
    pipelined copy-mode RC4 event loop.  The batcher's Create used to clear the state table on the
    default stream behind that work, after Enable had uploaded the states (GetState read zeros)."""
    torch = torch_dev
    n, L = 65536, 1500
    data = torch.from_numpy(workload.gen_records(0x5EED0002, 0, n, L)).cuda()
    offs = torch.arange(n, dtype=torch.int64, device="cuda") * L
    lens = torch.full((n,), L, dtype=torch.int32, device="cuda")
    keys = [bytes([k & 255, k >> 8]) * 8 for k in range(n)]
    st = torch.from_numpy(brb.rc4_states(keys)).cuda()
    Lb = brb.lib()
    s = torch.cuda.current_stream().cuda_stream
    flags = brb.BATCH_DEVICE | brb.BATCH_ASYNC
    for _ in range(4):
        assert Lb.BRB_RC4_CryptBatch(st.data_ptr(), data.data_ptr(), data.data_ptr(), offs.data_ptr(),
                                     lens.data_ptr(), n, flags, s) == 1
    T = 4 * ((L + 2) // 3)
    toffs = torch.arange(n, dtype=torch.int64, device="cuda") * T
    text = torch.zeros(n * T, dtype=torch.uint8, device="cuda")
    assert Lb.BRB_Base64EncodeBatch(data.data_ptr(), offs.data_ptr(), lens.data_ptr(), n, text.data_ptr(),
                                    toffs.data_ptr(), flags, s) == 1
    _event_loop(brb, orc, 1, False, True)
    torch.cuda.synchronize()


def _event_loop(brb, orc, algo, zero_copy, pipelined, seed=None, rounds=6):
    rng = np.random.default_rng(algo if seed is None else seed)
    C = 300
    keys = [rng.integers(0, 256, int(rng.integers(4, 32)), dtype=np.uint8).tobytes() for _ in range(C)]
    b = brb.TransformBatcher(C, 8 << 20, algo, zero_copy=zero_copy, pipelined=pipelined)
    pending = None
    ours_r = [orc.rc4_init(k) for k in keys]      # oracle model of the batcher's read states
    ours_w = [orc.rc4_init(k) for k in keys]      # ... and write states
    peer_w = [orc.rc4_init(k) for k in keys]      # the peer's write side (produces what we read)
    peer_r = [orc.rc4_init(k) for k in keys]      # the peer's read side (consumes what we write)
    for c in range(C):
        b.enable(c, keys[c])
    for rnd in range(rounds):
        expect = []
        for c in rng.permutation(C)[: int(rng.integers(C // 3, C))]:
            c = int(c)
            for _ in range(int(rng.integers(0, 4))):      # received buffers, in order
                n = int(rng.choice([0, 1, 5, 29, 64, 100, 1500, 4000]))
                payload = workload.gen_records(0x5EED00F2 + rnd, c * 16 + len(expect), 1, n).tobytes() if n else b""
                if algo == 2:
                    peer_w[c], frame = orc.rc4md5_frame(peer_w[c], payload, rnd * 1000 + c)
                    if rng.random() < 0.1 and len(frame) > 31:
                        frame = bytearray(frame)
                        frame[int(rng.integers(8, len(frame)))] ^= 4      # tampered on the wire
                        frame = bytes(frame)
                    ours_r[c], dec, ok = orc.rc4md5_open(ours_r[c], frame)
                    expect.append((c, 0, dec, ok))
                    assert b.read(c, frame) == 1
                else:
                    peer_w[c], wire = orc.rc4_crypt(peer_w[c], payload)
                    ours_r[c], dec = orc.rc4_crypt(ours_r[c], wire)
                    expect.append((c, 0, dec, 1))
                    assert b.read(c, wire) == 1
            for _ in range(int(rng.integers(0, 3))):      # outgoing buffers, in order
                n = int(rng.choice([0, 3, 77, 1500]))
                payload = workload.gen_records(0x5EED00F3 + rnd, c * 16 + len(expect), 1, n).tobytes() if n else b""
                salt = int(rng.integers(0, 2**32))
                if algo == 2:
                    ours_w[c], frame = orc.rc4md5_frame(ours_w[c], payload, salt)
                    peer_r[c], dec, ok = orc.rc4md5_open(peer_r[c], frame)
                    assert ok == 1 and dec[30:] == payload
                    expect.append((c, 1, frame, 1))
                else:
                    ours_w[c], wire = orc.rc4_crypt(ours_w[c], payload)
                    expect.append((c, 1, wire, 1))
                assert b.write(c, payload, salt) == 1
        if pipelined:
            got = b.flush_async()
            if pending is None:
                assert got == []
            else:
                _check_round(got, pending, rnd - 1)
            pending = expect
        else:
            _check_round(b.flush(), expect, rnd)
        for c in range(0, C, 7):     # GetState waits for the stream: the running round is included
            assert b.state(c, 0) == ours_r[c] and b.state(c, 1) == ours_w[c]
    if pipelined:
        _check_round(b.flush(), pending, rounds - 1)
        assert b.flush() == [] and b.flush_async() == []
    b.close()


def test_round_full_and_bad_args(brb, torch_dev):
    b = brb.TransformBatcher(2, 1000, 2)
    with pytest.raises(RuntimeError):
        b.enable(5, b"k")                         # connection id out of range
    b.enable(0, b"key")
    assert b.read(1, b"x") == -1                 # not enabled
    assert b.read(0, bytes(600)) == 1
    assert b.read(0, bytes(600)) == 0            # round full: flush first
    assert len(b.flush()) == 1
    assert b.read(0, bytes(600)) == 1
    for _ in range(7):
        b.write(0, b"", 0)
    assert b.write(0, b"", 0) == 0               # 4 buffers per connection on average
    assert len(b.flush()) == 8
    b.close()


def test_zero_copy_needs_page_locked(brb, orc, torch_dev):
    """Zero-copy rounds refuse a buffer outside page-locked memory and take one inside a region
    registered with BRB_CryptoGPU_HostRegister (also at an odd offset)."""
    import ctypes
    L = brb.lib()
    h = L.BRB_TransformBatcherCreate(4, 1 << 16, 1 | brb.BATCHER_ZERO_COPY)
    assert h
    try:
        assert L.BRB_TransformBatcherEnable(h, 0, b"key", 3) == 1
        plain = ctypes.create_string_buffer(b"pageable", 8)
        assert L.BRB_TransformBatcherRead(h, 0, plain, 8) == -1
        assert b"page-locked" in L.BRB_CryptoGPU_LastError()
        reg = brb.crypto.HostRegion(8192)
        ctypes.memmove(reg.addr + 3, b"in place", 8)
        assert L.BRB_TransformBatcherRead(h, 0, reg.addr + 3, 8) == 1
        got = []
        fn = brb.crypto.TransformDone(lambda _u, c, op, out, n, v: got.append(ctypes.string_at(out, n)))
        assert L.BRB_TransformBatcherFlush(h, fn, None) == 1
        assert got == [orc.rc4_crypt(orc.rc4_init(b"key"), b"in place")[1]]
        assert ctypes.string_at(reg.addr + 3, 8) == b"in place"    # input untouched
        reg.close()
        assert L.BRB_CryptoGPU_HostUnregister(ctypes.c_void_p(reg.addr)) == -1
    finally:
        L.BRB_TransformBatcherDestroy(h)


@pytest.mark.parametrize("pipelined", [False, True])
def test_concurrent_submitters(brb, orc, torch_dev, pipelined):
    """Several event threads (the reference's mt_engine, ev_kq_base.c:95) submit into one round at
    once, each owning its connections; every connection's results must come back in its own order
    and equal the oracle's per-buffer hook.  ctypes releases the GIL, so the Read/Write calls run
    concurrently."""
    import threading
    T, C, rounds = 4, 64, 4
    rng = np.random.default_rng(7)
    keys = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(C)]
    b = brb.TransformBatcher(C, 16 << 20, 2, pipelined=pipelined)
    for c in range(C):
        b.enable(c, keys[c])
    ours_r = [orc.rc4_init(k) for k in keys]
    ours_w = [orc.rc4_init(k) for k in keys]
    peer_w = [orc.rc4_init(k) for k in keys]
    want = {c: [] for c in range(C)}
    got = {c: [] for c in range(C)}
    for rnd in range(rounds):
        work = {t: [] for t in range(T)}          # per thread, in its submission order
        for c in range(C):
            for k in range(3):
                payload = workload.gen_records(0x5EED00F4 + rnd, c * 8 + k, 1, 1 + (c * 37 + k * 101) % 1600).tobytes()
                if k % 2 == 0:
                    peer_w[c], frame = orc.rc4md5_frame(peer_w[c], payload, rnd * 100 + c)
                    ours_r[c], dec, ok = orc.rc4md5_open(ours_r[c], frame)
                    want[c].append((0, dec, ok))
                    work[c % T].append(("r", c, frame))
                else:
                    ours_w[c], frame = orc.rc4md5_frame(ours_w[c], payload, k)
                    want[c].append((1, frame, 1))
                    work[c % T].append(("w", c, payload, k))
        rcs = []

        def run(t):
            for item in work[t]:
                rcs.append(b.read(item[1], item[2]) if item[0] == "r" else b.write(item[1], item[2], item[3]))

        ths = [threading.Thread(target=run, args=(t,)) for t in range(T)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        assert rcs == [1] * (3 * C)
        res = b.flush_async() if pipelined else b.flush()
        for conn, op, out, valid in res:
            got[conn].append((op, out, valid))
    for conn, op, out, valid in b.flush():
        got[conn].append((op, out, valid))
    for c in range(C):
        assert got[c] == want[c], c
        assert b.state(c, 0) == ours_r[c] and b.state(c, 1) == ours_w[c]
    b.close()


def test_pipelined_edges(brb, orc, torch_dev):
    """FlushAsync without BRB_BATCHER_PIPELINED is Flush; an empty FlushAsync delivers the running
    round; a full round still reports 0 and keeps its buffers; Destroy with a round still running
    waits for it (its results are dropped) instead of freeing memory the GPU is using."""
    key = b"edge-key"
    plain = brb.TransformBatcher(1, 4096, 1)
    plain.enable(0, key)
    assert plain.read(0, b"abc") == 1
    assert [r[2] for r in plain.flush_async()] == [orc.rc4_crypt(orc.rc4_init(key), b"abc")[1]]
    plain.close()

    b = brb.TransformBatcher(1, 1000, 1, pipelined=True)
    b.enable(0, key)
    st = orc.rc4_init(key)
    assert b.read(0, bytes(600)) == 1
    assert b.read(0, bytes(600)) == 0            # round full: flush first
    assert b.flush_async() == []                 # round 1 runs
    assert b.read(0, bytes(600)) == 1            # round 2 fills the other arena
    got1 = b.flush_async()                       # round 2 runs, round 1 delivered
    st, want1 = orc.rc4_crypt(st, bytes(600))
    assert [r[2] for r in got1] == [want1]
    assert [r[2] for r in b.flush_async()] == [orc.rc4_crypt(st, bytes(600))[1]]   # nothing new
    assert b.flush() == [] and b.flush_async() == []
    assert b.read(0, b"left running") == 1
    assert b.flush_async() == []
    b.close()                                    # waits for the running round


def test_failed_round_is_dropped_once(brb, orc, torch_dev):
    """A round whose enqueue fails part-way is dropped, never re-run (transform_batcher.hip
    launch_round).  BRB_TransformBatcherInjectFault(b, 1) makes the second kernel launch of a round
    report a failure without running: connection 0 has two read buffers (sub-rounds 0 and 1), so
    group 0 (its first buffer) runs and group 1 does not.  Flush returns BRB_BATCH_DROPPED with the
    reason, and both buffers' callbacks fire with valid = BRB_TRANSFORM_DROPPED and no output; the
    next Flush has nothing to run; the state shows the first buffer applied exactly once."""
    b = brb.TransformBatcher(4, 1 << 20, 1)
    b.inject_fault(1)
    key = b"faultkey"
    b.enable(0, key)
    st = orc.rc4_init(key)
    first = bytes(range(200))
    assert b.read(0, first) == 1 and b.read(0, bytes(100)) == 1
    with pytest.raises(RuntimeError, match="dropped") as ei:
        b.flush()
    assert ei.value.results == [(0, 0, b"", brb.TRANSFORM_DROPPED)] * 2
    b.inject_fault(-1)
    assert b.flush() == []                         # the failed round is gone, nothing re-runs
    st_once, _ = orc.rc4_crypt(st, first)
    assert b.state(0, 0) == st_once                # group 0 ran once; group 1 never ran
    # the batcher keeps working: the next buffer continues from that state
    assert b.read(0, first) == 1
    got = b.flush()
    st_twice, want = orc.rc4_crypt(st_once, first)
    assert got == [(0, 0, want, 1)] and b.state(0, 0) == st_twice
    b.close()


def test_pipelined_drop_keeps_delivered_round(brb, orc, torch_dev):
    """Pipelined Flush delivers the round FlushAsync left running, then the current round fails:
    the delivered round's results still come back through their callbacks, the dropped buffers'
    callbacks carry BRB_TRANSFORM_DROPPED, and the call returns BRB_BATCH_DROPPED (not 0)."""
    key = b"pipe-drop"
    b = brb.TransformBatcher(2, 1 << 16, 1, pipelined=True)
    b.enable(0, key)
    st = orc.rc4_init(key)
    assert b.read(0, b"first round") == 1
    assert b.flush_async() == []                   # round 1 runs
    b.inject_fault(0)                              # every launch of the next round fails
    assert b.read(0, b"second round") == 1
    with pytest.raises(RuntimeError, match="dropped") as ei:
        b.flush()
    st, want = orc.rc4_crypt(st, b"first round")
    assert ei.value.results == [(0, 0, want, 1), (0, 0, b"", brb.TRANSFORM_DROPPED)]
    assert b.state(0, 0) == st
    b.close()


def test_states_survive_busy_default_stream(brb, orc, torch_dev):
    """Regression (round-3 cause of the all-zero RC4 state): Create zeroed the state
    table with hipMemset, i.e. on the legacy default stream, which the batcher's non-blocking stream
    does not wait for.  With the default stream busy (a long kernel queued on it first), that memset
    ran after Enable's state uploads and after the first round, and GetState read zeros.  The table
    is now cleared on the batcher's own stream before Create returns."""
    torch = torch_dev
    key = b"busy-default-stream"
    torch.cuda._sleep(200_000_000)                # ~0.1 s of spinning on the default stream
    b = brb.TransformBatcher(4, 1 << 16, 1, pipelined=True)
    b.enable(0, key)
    st = orc.rc4_init(key)
    assert b.read(0, b"hello, busy stream") == 1
    assert b.flush_async() == []
    st, want = orc.rc4_crypt(st, b"hello, busy stream")
    assert b.flush() == [(0, 0, want, 1)]
    torch.cuda.synchronize()                       # the default stream's work has all landed
    assert b.state(0, 0) == st and b.state(0, 1) == orc.rc4_init(key)
    b.close()


@pytest.mark.parametrize("all_devices", [False, True])
@pytest.mark.parametrize("pipelined", [False, True])
@pytest.mark.parametrize("zero_copy", [False, True])
@pytest.mark.parametrize("algo", [1, 2])
def test_pair_fault_round_dropped(brb, orc, torch_dev, algo, zero_copy, pipelined, all_devices):
    """A wave-pair protocol fault inside a batcher round (test option pair_stall, on the pair kernels
    the rounds run: the RC4 pass, the RC4+MD5 frame and open) drops the round: every buffer comes
    back with valid = BRB_TRANSFORM_DROPPED and no output, Flush returns BRB_BATCH_DROPPED -- no
    plaintext, frame or valid flag computed over wrong bytes is delivered (ev_kq_aio_transform.c:
    157-184 must never pass over them).  After re-keying (Enable) the next round equals the oracle.
    all_devices: BRB_BATCHER_ALL_DEVICES forced into two parts (test option "devices"): every part's
    round is dropped (callbacks come part by part, so results are compared as sets of (conn, op):
    one buffer per connection and direction here)."""
    rng = np.random.default_rng(100 + algo)
    C = 192                                       # > 64 per part: the stalled wave's group and ordinary ones
    keys = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(C)]
    with brb.TestOption("devices", 2 if all_devices else 0):
        b = brb.TransformBatcher(C, 4 << 20, algo, zero_copy=zero_copy, pipelined=pipelined, all_devices=all_devices)
    same = (lambda x, y: sorted(x) == sorted(y)) if all_devices else (lambda x, y: x == y)

    def rekey():
        for c in range(C):
            b.enable(c, keys[c])
        return ([orc.rc4_init(k) for k in keys], [orc.rc4_init(k) for k in keys], [orc.rc4_init(k) for k in keys])

    def submit(rnd, ours_r, ours_w, peer_w):
        expect = []
        for c in range(C):
            n = int(rng.choice([0, 17, 700, 1500, 3000]))
            payload = workload.gen_records(0x5EED00F6 + rnd, c, 1, n).tobytes() if n else b""
            if algo == 2:
                peer_w[c], frame = orc.rc4md5_frame(peer_w[c], payload, c)
                ours_r[c], dec, ok = orc.rc4md5_open(ours_r[c], frame)
                expect.append((c, 0, dec, ok))
                assert b.read(c, frame) == 1
                ours_w[c], out = orc.rc4md5_frame(ours_w[c], payload, rnd + c)
            else:
                peer_w[c], wire = orc.rc4_crypt(peer_w[c], payload)
                ours_r[c], dec = orc.rc4_crypt(ours_r[c], wire)
                expect.append((c, 0, dec, 1))
                assert b.read(c, wire) == 1
                ours_w[c], out = orc.rc4_crypt(ours_w[c], payload)
            expect.append((c, 1, out, 1))
            assert b.write(c, payload, rnd + c) == 1
        return expect

    ours_r, ours_w, peer_w = rekey()
    expect = submit(0, ours_r, ours_w, peer_w)
    dropped = [(c, op, b"", brb.TRANSFORM_DROPPED) for c, op, _, _ in expect]
    with brb.TestOption("rc4_pair", 1), brb.TestOption("rc4md5_pair", 1), brb.TestOption("pair_stall", 1):
        if pipelined:
            assert b.flush_async() == []          # launched with the stalled kernels, not delivered
        else:
            with pytest.raises(RuntimeError, match="wave-pair protocol fault.*dropped") as ei:
                b.flush()
    if pipelined:
        with pytest.raises(RuntimeError, match="wave-pair protocol fault.*dropped") as ei:
            b.flush()
    assert ei.value.code == brb.BATCH_DROPPED
    assert same(ei.value.results, dropped)
    assert b.flush() == []                        # the dropped round is gone, nothing re-runs
    ours_r, ours_w, peer_w = rekey()              # its connections are re-keyed, as after a lost buffer
    expect = submit(1, ours_r, ours_w, peer_w)
    got = b.flush()
    if all_devices:
        assert same(got, expect)
    else:
        _check_round(got, expect, 1)
    for c in range(0, C, 5):
        assert b.state(c, 0) == ours_r[c] and b.state(c, 1) == ours_w[c]
    b.close()


@pytest.mark.parametrize("how", ["async", "sync"])
@pytest.mark.parametrize("zero_copy", [False, True])
@pytest.mark.parametrize("algo", [1, 2])
def test_pipelined_fault_poisons_next_round(brb, orc, torch_dev, algo, zero_copy, how):
    """on a pipelined batcher, round A runs with a wave-pair fault (test option
    pair_stall) while round B is submitted behind it.  A's connections are poisoned when A is
    dropped, so none of B's buffers on them is delivered as data -- with "async" B is launched by the
    FlushAsync that finds A's fault (B ran on the wrong states: dropped at delivery); with "sync"
    Flush finds the fault before launching B (B's buffers on those connections never run).
    Connections A did not touch are delivered normally throughout.  Read/Write refuse a poisoned
    connection until Enable re-keys it; then every connection equals the oracle again."""
    rng = np.random.default_rng(300 + algo)
    C, CA = 192, 160                              # round A holds connections 0..CA-1
    keys = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(C)]
    b = brb.TransformBatcher(C, 4 << 20, algo, zero_copy=zero_copy, pipelined=True)
    st = {}

    def rekey(conns):
        for c in conns:
            b.enable(c, keys[c])
            st[c] = [orc.rc4_init(keys[c]) for _ in range(3)]   # ours read, ours write, peer write

    def submit(c, rnd):
        """one read and one write on connection c; returns their expected callbacks"""
        n = int(rng.choice([0, 17, 700, 1500]))
        payload = workload.gen_records(0x5EED00F8 + rnd, c, 1, n).tobytes() if n else b""
        r, w, pw = st[c]
        if algo == 2:
            pw, frame = orc.rc4md5_frame(pw, payload, c)
            r, dec, ok = orc.rc4md5_open(r, frame)
            assert b.read(c, frame) == 1
            w, out = orc.rc4md5_frame(w, payload, rnd + c)
            exp = [(c, 0, dec, ok), (c, 1, out, 1)]
        else:
            pw, wire = orc.rc4_crypt(pw, payload)
            r, dec = orc.rc4_crypt(r, wire)
            assert b.read(c, wire) == 1
            w, out = orc.rc4_crypt(w, payload)
            exp = [(c, 0, dec, 1), (c, 1, out, 1)]
        assert b.write(c, payload, rnd + c) == 1
        st[c] = [r, w, pw]
        return exp

    def dropped(c):
        return [(c, 0, b"", brb.TRANSFORM_DROPPED), (c, 1, b"", brb.TRANSFORM_DROPPED)]

    rekey(range(C))
    for c in range(CA):
        submit(c, 0)
    with brb.TestOption("rc4_pair", 1), brb.TestOption("rc4md5_pair", 1), brb.TestOption("pair_stall", 1):
        assert b.flush_async() == []              # A launched with the stalled kernels
    want_b = []
    for c in range(C):                            # B: every connection, submitted before A's fault is known
        e = submit(c, 1)
        want_b += dropped(c) if c < CA else e
    want_a = [x for c in range(CA) for x in dropped(c)]
    if how == "async":
        with pytest.raises(RuntimeError, match="wave-pair protocol fault.*dropped") as ei:
            b.flush_async()                       # launches B, then delivers (drops) A
        assert ei.value.code == brb.BATCH_DROPPED and ei.value.results == want_a
        assert b.read(0, b"refused") == -1 and b.write(CA - 1, b"refused", 0) == -1
        want_c = submit(CA, 2)                    # an untouched connection keeps working
        with pytest.raises(RuntimeError, match="out of step.*dropped") as ei:
            b.flush()                             # delivers B (poisoned buffers dropped), then C
        assert ei.value.code == brb.BATCH_DROPPED
        _check_round(ei.value.results, want_b + want_c, 1)
    else:
        with pytest.raises(RuntimeError, match="dropped") as ei:
            b.flush()                             # delivers (drops) A, then runs B without its stale buffers
        assert ei.value.code == brb.BATCH_DROPPED
        _check_round(ei.value.results, want_a + want_b, 1)
        assert b.read(0, b"refused") == -1
    for c in range(CA, C, 7):                     # untouched connections: their states advanced exactly once
        assert b.state(c, 0) == st[c][0] and b.state(c, 1) == st[c][1]
    rekey(range(CA))                              # A's connections re-keyed, as after a lost buffer
    want_d = [x for c in range(C) for x in submit(c, 3)]
    _check_round(b.flush(), want_d, 3)
    for c in range(0, C, 5):
        assert b.state(c, 0) == st[c][0] and b.state(c, 1) == st[c][1]
    b.close()
