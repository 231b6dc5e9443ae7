"""MemBuffer Blowfish: BRB_MemBufferEncrypt / BRB_MemBufferDecrypt against the
oracle's restatement of mem_buf.c:1499-1617 (pinned by tests/golden/quirks.json), with its quirks:
keyLen 4 on encrypt vs 64 on decrypt, the +2 padding words, the zero-word stop, the size rules."""
import numpy as np
import pytest

from brb_framework_amd import workload


def test_key_matches_oracle(brb, orc, golden):
    assert brb.membuf_key(0x4FD9).hex() == golden["quirks"]["membuf_key_4fd9"]
    for seed in (0, 1, 7, 0x4FD9, 0xFFFFFFFF, 123456789):
        assert brb.membuf_key(seed) == orc.membuf_key(seed)


def test_span_macro(brb):
    for data_size in range(0, 140):
        words = data_size // 8 + 2                       # mem_buf.c:1504 + :1518 ("+2" padding)
        assert brb.membuf_span(data_size) == 16 * ((words + 1) // 2)


@pytest.fixture(scope="module")
def torch_dev(brb):
    import torch
    assert torch.cuda.is_available(), "no HIP device visible to torch"
    assert brb.gpu_available(), brb.lib().BRB_CryptoGPU_LastError()
    return torch


def _buf(size, off, seed):
    raw = workload.gen_records(seed, 3, 1, size) if size else np.zeros(0, np.uint8)
    need = off + (((size + off) // 8 + 4) // 2) * 16 + 16
    b = np.zeros(need, np.uint8)
    b[:size] = raw
    return b


@pytest.mark.gpu
def test_golden_membuffer_cases(brb, golden):
    for c in golden["quirks"]["membuffer"]:
        plain = np.frombuffer(bytes.fromhex(c["plain"]), np.uint8)
        buf = np.zeros(plain.size + 64, np.uint8)
        buf[: plain.size] = plain
        ns = brb.membuf_encrypt(buf, c["size"], c["seed"], c["offset"])
        assert ns == c["enc_size"]
        assert buf[: len(c["enc"]) // 2].tobytes().hex() == c["enc"]
        ds = brb.membuf_decrypt(buf, ns, c["seed"], c["offset"])
        assert ds == c["dec_size"]
        assert buf[: len(c["dec"]) // 2].tobytes().hex() == c["dec"]


@pytest.mark.gpu
@pytest.mark.parametrize("off", [0, 1, 5, 8, 16, 24])
@pytest.mark.parametrize("size", [0, 1, 7, 8, 9, 15, 16, 17, 100, 1023, 4096, 100003])
def test_membuffer_vs_oracle(brb, orc, torch_dev, size, off):
    seed = 0x4FD9 + size + off
    b = _buf(size, off, seed)
    want = b.copy()
    ns_want = orc.membuf_encrypt(bytearray_view := bytearray(want.tobytes()), size, seed, off)
    want = np.frombuffer(bytes(bytearray_view), np.uint8).copy()
    host = b.copy()
    assert brb.membuf_encrypt(host, size, seed, off) == ns_want
    assert np.array_equal(host, want)
    if off % 8 == 0:                       # device mode needs buf + offset 8-byte aligned
        d = torch_dev.from_numpy(b.copy()).cuda()
        assert brb.membuf_encrypt(d, size, seed, off) == ns_want
        assert np.array_equal(d.cpu().numpy(), want)
    # decrypt of the ciphertext (the reference's keyLen-64 quirk: not the plaintext)
    dec_want = bytearray(want.tobytes())
    ds_want = orc.membuf_decrypt(dec_want, ns_want, seed, off)
    dec = want.copy()
    assert brb.membuf_decrypt(dec, ns_want, seed, off) == ds_want
    assert dec.tobytes() == bytes(dec_want)


@pytest.mark.gpu
@pytest.mark.parametrize("zero_at", [0, 1, 2, 77, 500, 1023])
def test_decrypt_stops_at_zero_pair(brb, orc, torch_dev, zero_at):
    size, seed = 16 * 1024, 99
    b = _buf(size, 0, seed)
    w = b[: 16 * 1024].view(np.uint64)
    w[w == 0] = 1
    w[2 * zero_at + (zero_at & 1)] = 0             # a zero xl or xr in pair zero_at
    want = bytearray(b.tobytes())
    ds_want = orc.membuf_decrypt(want, size, seed, 0)
    assert ds_want == 16 * zero_at
    d = torch_dev.from_numpy(b.copy()).cuda()
    assert brb.membuf_decrypt(d, size, seed, 0) == ds_want
    assert d.cpu().numpy().tobytes() == bytes(want)
    h = b.copy()
    assert brb.membuf_decrypt(h, size, seed, 0) == ds_want and h.tobytes() == bytes(want)


@pytest.mark.gpu
def test_membuffer_rejects(brb, torch_dev):
    d = torch_dev.zeros(256, dtype=torch_dev.uint8, device="cuda")
    with pytest.raises(RuntimeError):
        brb.membuf_encrypt(d, 10, 1, offset=3)     # unaligned device words
    h = np.zeros(256, np.uint8)
    with pytest.raises((RuntimeError, ValueError)):
        brb.membuf_decrypt(h, 4, 1, offset=8)      # size < offset


@pytest.mark.gpu
@pytest.mark.parametrize("without_quotes", [False, True])
def test_kv_file_round_trip(brb, orc, torch_dev, tmp_path, without_quotes):
    """Encrypted K/V files (key_value.c:464-506): the written bytes are the oracle's
    MemBufferEncryptData(text, KV_SEED, 0), and reading gives the oracle's MemBufferDecryptData of
    them (not the text: the reference's keyLen 4/64 asymmetry)."""
    from brb_framework_amd import kv
    pairs = [("listen_port", "8080"), ("name", "brb"), (None, "x"), ("path", "/var/lib/brb/" + "d" * 77),
             ("empty", "")] + [(f"k{i}", str(i * 7919)) for i in range(40)]
    text = kv.kv_assemble(pairs, without_quotes)
    assert text.startswith(b"listen_port=8080\n" if without_quotes else b'listen_port="8080"\n')
    p = tmp_path / "brb.conf"
    assert kv.kv_write_file(p, pairs, enc=True, without_quotes=without_quotes) == 1
    buf = bytearray(text) + bytearray(brb.membuf_span(len(text)) + 16)
    n = orc.membuf_encrypt(buf, len(text), kv.KV_SEED, 0)
    want = bytes(buf[:n])
    assert p.read_bytes() == want
    dbuf = bytearray(want) + bytearray(brb.membuf_span(len(want)) + 16)
    dn = orc.membuf_decrypt(dbuf, len(want), kv.KV_SEED, 0)
    assert kv.kv_read_file(p) == bytes(dbuf[:dn])
    q = tmp_path / "plain.conf"
    kv.kv_write_file(q, pairs, enc=False, without_quotes=without_quotes)
    assert kv.kv_read_file(q, enc=False) == text
