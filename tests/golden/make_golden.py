#!/usr/bin/env python3
"""Generate tests/golden/*.json -- the fixtures that pin the oracle and the GPU path.

Sources, in order of authority (DESIGN.md "Oracle"):
  * published known answers typed in from their standards: RFC 1321 A.5 (MD5), FIPS 180-1
    appendices A/B/C (SHA-1), Kocher's Blowfish self-test ("TESTKEY") and Eric Young's Blowfish ECB
    vectors.  Each is re-checked here against an independent implementation before it is written
    (hashlib for MD5/SHA-1, OpenSSL libcrypto BF_ecb_encrypt for Blowfish).
  * Python hashlib (OpenSSL) digests of the SURVEY §8(d) generator at the edge lengths and of the
    first/last records of configs 1-3.  The survey verified BRB_MD5*/BrbSha1_* == hashlib on 20 edge
    lengths with the reference compiled in its container.
  * the oracle restatement (oracle/brb_oracle.c) for what no external source pins: the HIGH 32 bits
    of the reference's 64-bit Blowfish words, the SHA-1 in-place mutation bytes and the MemBuffer
    wrappers.  These are marked "source": "oracle" -- regression fixtures, not pins.
  * for the 64-bit Blowfish words, a second, independent derivation written here: Python big
    integers reduced mod 2^64 (the LP64 `unsigned long` of blowfish.c:312-462), with the pi tables
    computed by the Chudnovsky series (the oracle uses BBP digit extraction, the product's header
    Machin's formula).  blowfish64.json is written only if both derivations agree on every word.

The reference itself cannot be built here (libbrb_data.h needs <bsd/string.h>, absent; stand-in
headers are not allowed), so no fixture comes from running reference code.

Usage (in the repo root):  python tests/golden/make_golden.py
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from brb_framework_amd import workload  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))

MD5_KAT = [  # RFC 1321 appendix A.5
    ("", "d41d8cd98f00b204e9800998ecf8427e"),
    ("a", "0cc175b9c0f1b6a831c399e269772661"),
    ("abc", "900150983cd24fb0d6963f7d28e17f72"),
    ("message digest", "f96b697d7cb7938d525a2f31aaf161d0"),
    ("abcdefghijklmnopqrstuvwxyz", "c3fcd3d76192e4007dfb496cca67e13b"),
    ("ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789", "d174ab98d277d9f5a5611c2c9f419d9f"),
    ("1234567890" * 8, "57edf4a22be3c955ac49da2e2107b67a"),
]
SHA1_KAT = [  # FIPS 180-1 appendices A, B, C
    ("abc", 1, "a9993e364706816aba3e25717850c26c9cd0d89d"),
    ("abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq", 1, "84983e441c3bd26ebaae4aa1f95129e5e54670f1"),
    ("a", 1000000, "34aa973cd4c4daa4f61eeb2bdbad27316534016f"),
]
BF_KAT = [  # (key hex, plaintext hex, ciphertext hex); Eric Young's ECB set + Kocher's self-test
    ("0000000000000000", "0000000000000000", "4EF997456198DD78"),
    ("FFFFFFFFFFFFFFFF", "FFFFFFFFFFFFFFFF", "51866FD5B85ECB8A"),
    ("3000000000000000", "1000000000000001", "7D856F9A613063F2"),
    ("1111111111111111", "1111111111111111", "2466DD878B963C9D"),
    ("0123456789ABCDEF", "1111111111111111", "61F9C3802281B096"),
    ("1111111111111111", "0123456789ABCDEF", "7D0CC630AFDA1EC7"),
    ("FEDCBA9876543210", "0123456789ABCDEF", "0ACEAB0FC6A0A28D"),
    ("7CA110454A1A6E57", "01A1D6D039776742", "59C68245EB05282B"),
    ("0131D9619DC1376E", "5CD54CA83DEF57DA", "B1B8CC0B250F09A0"),
    ("544553544B4559", "0000000100000002", "DF333FD230A71BB4"),          # "TESTKEY", (1, 2)
    ("6162636465666768696A6B6C6D6E6F707172737475767778797A", "424C4F5746495348", "324ED0FEF413A203"),
]
EDGE_LENGTHS = [0, 1, 3, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 129, 1500, 16384, 65535, 65536, 65537]


def libcrypto_bf(key: bytes, pt: bytes) -> bytes:
    L = ctypes.CDLL("libcrypto.so.3")
    ks = ctypes.create_string_buffer(8192)
    L.BF_set_key(ks, len(key), key)
    out = ctypes.create_string_buffer(8)
    L.BF_ecb_encrypt(pt, out, ks, 1)
    return out.raw


RC4_KAT = [  # (key hex, plaintext hex, ciphertext hex): RFC 6229 section 2 (key 0x0102030405,
    # keystream offset 0) and the three classic vectors ("Key"/"Wiki"/"Secret")
    ("0102030405", "00" * 16, "b2396305f03dc027ccc3524a0a1118a8"),
    (b"Key".hex(), b"Plaintext".hex(), "bbf316e8d940af0ad3"),
    (b"Wiki".hex(), b"pedia".hex(), "1021bf0420"),
    (b"Secret".hex(), b"Attack at dawn".hex(), "45a01f645fc35b383552544b9bf5"),
]


def libcrypto_rc4(key: bytes, data: bytes) -> bytes:
    """OpenSSL's RC4 (RC4_set_key / RC4, libcrypto.so.3): an independent implementation."""
    L = ctypes.CDLL("libcrypto.so.3")
    ks = ctypes.create_string_buffer(2048)        # RC4_KEY = {uint x, y; uint data[256]}
    L.RC4_set_key(ks, len(key), key)
    out = ctypes.create_string_buffer(max(len(data), 1))
    L.RC4(ks, ctypes.c_size_t(len(data)), data, out)
    return out.raw[: len(data)]


# ---- independent big-integer restatement of blowfish.c (second derivation of the 64-bit words) ----
M64 = (1 << 64) - 1


def pi_words_chudnovsky(n_words: int) -> list:
    """The first n_words 32-bit words of pi's fractional part (0x243F6A88, ...), from the Chudnovsky
    series by binary splitting, in integers only."""
    bits = 32 * n_words + 64                     # 64 guard bits
    terms = (bits * 30103 // 100000) // 14 + 3   # each term adds ~14.18 decimal digits

    def split(a, b):
        if b - a == 1:
            if a == 0:
                p = q = 1
            else:
                p = (6 * a - 5) * (2 * a - 1) * (6 * a - 1)
                q = a * a * a * 10939058860032000
            t = p * (13591409 + 545140134 * a)
            return p, q, (-t if a & 1 else t)
        m = (a + b) // 2
        p1, q1, t1 = split(a, m)
        p2, q2, t2 = split(m, b)
        return p1 * p2, q1 * q2, q2 * t1 + p1 * t2

    import math
    _, q, t = split(0, terms)
    pi_scaled = q * 426880 * math.isqrt(10005 << (2 * bits)) // t      # pi * 2^bits
    frac = (pi_scaled - (3 << bits)) >> 64
    return [(frac >> (32 * (n_words - 1 - i))) & 0xFFFFFFFF for i in range(n_words)]


class BigIntBlowfish:
    """BRB_Blowfish_Init/Encrypt/Decrypt (blowfish.c:312-443) with _F (:445-462) on LP64 words:
    every `unsigned long` operation is a Python integer operation reduced mod 2^64."""

    PI = None

    def __init__(self, key: bytes, key_len: int | None = None):
        if BigIntBlowfish.PI is None:
            BigIntBlowfish.PI = pi_words_chudnovsky(18 + 4 * 256)
        pi = BigIntBlowfish.PI
        key_len = len(key) if key_len is None else key_len
        self.S = [list(pi[18 + 256 * i: 18 + 256 * (i + 1)]) for i in range(4)]
        self.P = []
        j = 0
        for i in range(18):
            data = 0
            for _ in range(4):
                data = ((data << 8) | key[j]) & M64
                j += 1
                if j >= key_len:
                    j = 0
            self.P.append(pi[i] ^ data)
        xl = xr = 0
        for i in range(0, 18, 2):
            xl, xr = self.encrypt(xl, xr)
            self.P[i], self.P[i + 1] = xl, xr
        for i in range(4):
            for j in range(0, 256, 2):
                xl, xr = self.encrypt(xl, xr)
                self.S[i][j], self.S[i][j + 1] = xl, xr

    def f(self, x: int) -> int:
        a, b, c, d = (x >> 24) & 0xFF, (x >> 16) & 0xFF, (x >> 8) & 0xFF, x & 0xFF
        y = (self.S[0][a] + self.S[1][b]) & M64
        y ^= self.S[2][c]
        return (y + self.S[3][d]) & M64

    def encrypt(self, xl: int, xr: int):
        for i in range(16):
            xl ^= self.P[i]
            xr ^= self.f(xl)
            xl, xr = xr, xl
        xl, xr = xr, xl
        return xl ^ self.P[17], xr ^ self.P[16]

    def decrypt(self, xl: int, xr: int):
        for i in range(17, 1, -1):
            xl ^= self.P[i]
            xr ^= self.f(xl)
            xl, xr = xr, xl
        xl, xr = xr, xl
        return xl ^ self.P[0], xr ^ self.P[1]

    def ctx_bytes(self) -> bytes:
        """The 8336-byte BRB_BLOWFISH_CTX image (LP64, little-endian)."""
        return b"".join(v.to_bytes(8, "little") for v in self.P + [w for row in self.S for w in row])


def check_blowfish64(bf: dict) -> None:
    """Asserts that the big-integer derivation reproduces every word of a blowfish64.json dict."""
    for c in bf["contexts"]:
        b = BigIntBlowfish(bytes.fromhex(c["key"]))
        assert hashlib.sha256(b.ctx_bytes()).hexdigest() == c["sha256"], c["key"]
        assert [hex(v) for v in b.P] == c["P"], c["key"]
        # the carries make most entries wider than 32 bits, "up to 50 significant
        # bits" for the keys the survey ran; a 56-byte key reaches 51.  Each context's measured
        # width is part of the fixture.
        words = b.P + [w for row in b.S for w in row]
        assert max(w.bit_length() for w in words) == c["max_bits"], c["key"]
        assert sum(1 for w in words if w >> 32) > len(words) // 2, c["key"]
    g = bf["cfg4"]
    b = BigIntBlowfish(bytes.fromhex(g["key"]))
    words = [int(v) for v in workload.gen_words(g["seed"], 2 * g["pairs"])]
    assert hashlib.sha256(np.array(words, np.uint64).tobytes()).hexdigest() == g["plain_sha256"]
    ct = []
    for i in range(g["pairs"]):
        xl, xr = b.encrypt(words[2 * i], words[2 * i + 1])
        assert b.decrypt(xl, xr) == (words[2 * i], words[2 * i + 1])
        ct += [xl, xr]
    assert hashlib.sha256(np.array(ct, np.uint64).tobytes()).hexdigest() == g["cipher_sha256"]
    assert [hex(v) for v in ct[:16]] == g["cipher_first8"]


# ---- second derivations of the other oracle-only fixtures (quirks.json) ----
M32 = 0xFFFFFFFF


class ByteArraySha1:
    """BrbSha1_Init/Update/Final (sha1.c:132-200) on a caller-owned bytearray, written from the
    reference text independently of the oracle: Transform (:75-130) works IN the 64 bytes it is
    given, blk0 (:46-47) stores each byte-swapped word back and blk (:49-50) stores W[i] over
    l[i & 15], so a block hashed straight from the caller's data (:157-158) is left holding
    W[64..79] as little-endian words.  count[0] is 32 bits and compared with the 64-bit len << 3
    (:152), the spurious carry for single updates of 2^29 bytes or more."""

    def __init__(self):
        self.state = [0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0]
        self.count = [0, 0]
        self.buffer = bytearray(64)

    def _transform(self, mem: bytearray, off: int) -> None:
        l = [int.from_bytes(mem[off + 4 * k: off + 4 * k + 4], "little") for k in range(16)]
        rol = lambda v, n: ((v << n) | (v >> (32 - n))) & M32
        a, b, c, d, e = self.state
        for i in range(80):
            if i < 16:
                l[i] = int.from_bytes(l[i].to_bytes(4, "little"), "big")       # blk0: byte swap in place
            else:
                l[i & 15] = rol(l[(i + 13) & 15] ^ l[(i + 8) & 15] ^ l[(i + 2) & 15] ^ l[i & 15], 1)
            if i < 20:
                f, k = (b & (c ^ d)) ^ d, 0x5A827999
            elif i < 40:
                f, k = b ^ c ^ d, 0x6ED9EBA1
            elif i < 60:
                f, k = ((b | c) & d) | (b & c), 0x8F1BBCDC
            else:
                f, k = b ^ c ^ d, 0xCA62C1D6
            e, d, c, b, a = d, c, rol(b, 30), a, (e + f + l[i & 15] + k + rol(a, 5)) & M32
        for k in range(16):
            mem[off + 4 * k: off + 4 * k + 4] = l[k].to_bytes(4, "little")
        self.state = [(x + y) & M32 for x, y in zip(self.state, (a, b, c, d, e))]

    def update(self, data: bytearray, length: int) -> None:
        j = (self.count[0] >> 3) & 63
        bits = length << 3                                  # size_t
        self.count[0] = (self.count[0] + bits) & M32
        if self.count[0] < bits:
            self.count[1] = (self.count[1] + 1) & M32
        self.count[1] = (self.count[1] + (length >> 29)) & M32
        if j + length > 63:
            i = 64 - j
            self.buffer[j:64] = data[:i]
            self._transform(self.buffer, 0)
            while i + 63 < length:
                self._transform(data, i)                    # in the caller's memory
                i += 64
            j = 0
        else:
            i = 0
        self.buffer[j:j + length - i] = data[i:length]

    def final(self) -> bytes:
        fc = bytes((self.count[0 if i >= 4 else 1] >> ((3 - (i & 3)) * 8)) & 255 for i in range(8))
        self.update(bytearray(b"\x80"), 1)
        while (self.count[0] & 504) != 448:
            self.update(bytearray(1), 1)
        self.update(bytearray(fc), 8)
        return b"".join(v.to_bytes(4, "big") for v in self.state)


def membuffer_key(seed: int) -> bytes:
    """The 16 unsigned ints of mem_buf.c:1511-1515 / 1565-1569 (seed carried from word to word)."""
    out, s = [], seed & M32
    for i in range(16):
        k = ((i + s) * s + 13 * i) & M32
        out.append(k)
        s = (k * s) & M32
    return b"".join(k.to_bytes(4, "little") for k in out)


def membuffer_crypt(buf: bytearray, size: int, seed: int, offset: int, decrypt: bool) -> int:
    """MemBufferEncryptData / MemBufferDecryptData (mem_buf.c:1499-1617) on an already grown,
    zero-filled buffer, on BigIntBlowfish: the key is used with keyLen sizeof(enc_key[16]) = 4 to
    encrypt and sizeof(enc_key) = 64 to decrypt; blocks = size / 8 + 2 words from byte `offset`;
    decryption stops at the first pair with a zero word.  Returns the new MemBuffer size."""
    key = membuffer_key(seed)
    bf = BigIntBlowfish(key, 64 if decrypt else 4)
    blocks = (size - offset if decrypt else size + offset) // 8 + 2
    word = lambda k: int.from_bytes(buf[offset + 8 * k: offset + 8 * k + 8], "little")
    i = 0
    while i < blocks:
        xl, xr = word(i), word(i + 1)
        if decrypt and (xl == 0 or xr == 0):
            break
        xl, xr = bf.decrypt(xl, xr) if decrypt else bf.encrypt(xl, xr)
        buf[offset + 8 * i: offset + 8 * i + 16] = xl.to_bytes(8, "little") + xr.to_bytes(8, "little")
        i += 2
    return i * 8 + offset


def check_quirks(q: dict) -> None:
    """Asserts that the second derivations above reproduce every byte of a quirks.json dict."""
    s = q["sha1_inplace"]
    msg = bytearray.fromhex(s["input"])
    h = ByteArraySha1()
    h.update(msg, len(msg))
    assert msg.hex() == s["after_update"]
    assert h.final().hex() == s["digest"] == s["hashlib_digest"]
    assert membuffer_key(0x4FD9).hex() == q["membuf_key_4fd9"]
    for m in q["membuffer"]:
        enc = bytearray.fromhex(m["plain"])
        assert membuffer_crypt(enc, m["size"], m["seed"], m["offset"], False) == m["enc_size"]
        assert enc.hex() == m["enc"]
        assert membuffer_crypt(enc, m["enc_size"], m["seed"], m["offset"], True) == m["dec_size"]
        assert enc.hex() == m["dec"]


def dump(name, obj):
    with open(os.path.join(OUT, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
        f.write("\n")


def main():
    # ---- published known answers, each cross-checked ----
    for m, d in MD5_KAT:
        assert hashlib.md5(m.encode()).hexdigest() == d, m
    for m, rep, d in SHA1_KAT:
        assert hashlib.sha1(m.encode() * rep).hexdigest() == d, m
    for k, p, c in BF_KAT:
        assert libcrypto_bf(bytes.fromhex(k), bytes.fromhex(p)).hex().upper() == c, k
    dump("kat.json", {
        "md5_rfc1321": [{"msg": m, "digest": d} for m, d in MD5_KAT],
        "sha1_fips180_1": [{"msg": m, "repeat": r, "digest": d} for m, r, d in SHA1_KAT],
        "blowfish_ecb": [{"key": k, "plain": p, "cipher": c} for k, p, c in BF_KAT],
        "note": "Blowfish vectors pin only the LOW 32 bits of each 64-bit reference word "
                "(the reference's xl/xr are unsigned long; blowfish.c:445-462 keeps carries in the high half).",
    })

    # ---- generator digests (hashlib) ----
    seed = workload.SEEDS[1]
    edge = []
    for n in EDGE_LENGTHS:
        rec = workload.gen_records(seed, 7, 1, n).tobytes()
        edge.append({"len": n, "record": 7, "md5": hashlib.md5(rec).hexdigest(),
                     "sha1": hashlib.sha1(rec).hexdigest(), "first8": rec[:8].hex()})
    cfgs = {}
    for c in (1, 2, 3, 5):
        cfg = workload.CONFIGS[c]
        n, L = cfg["records"], cfg["rec_len"]
        idx = set(list(range(min(64, n))) + list(range(max(0, n - 64), n)))
        if c == 5:   # both ends of every GPU's shard: records [g N/8, (g+1) N/8)
            for g in range(8):
                r0, r1 = workload.shard(n, g, 8)
                idx |= {r0, r0 + 1, r1 - 2, r1 - 1}
        idx = sorted(idx)
        recs = []
        for r in idx:
            b = workload.gen_records(workload.SEEDS[c], r, 1, L).tobytes()
            recs.append({"r": r, "md5": hashlib.md5(b).hexdigest(), "sha1": hashlib.sha1(b).hexdigest()})
        cfgs[str(c)] = {"seed": workload.SEEDS[c], "records": n, "rec_len": L, "digests": recs}
    dump("digests.json", {"source": "hashlib (OpenSSL 3) over the SURVEY §8(d) generator",
                          "generator_seed": seed, "edge": edge, "configs": cfgs})

    # ---- oracle-only regression fixtures (64-bit Blowfish, SHA-1 mutation, MemBuffer) ----
    bf = {"source": "oracle", "contexts": [], "cfg4": {}}
    for key in (b"TESTKEY", workload.CFG4_KEY, bytes(range(56))):
        c = oracle.bf_init(key)
        raw = oracle.bf_ctx_bytes(c)
        words = list(c.P) + [c.S[i][j] for i in range(4) for j in range(256)]
        bf["contexts"].append({"key": key.hex(), "sha256": hashlib.sha256(raw).hexdigest(),
                               "max_bits": max(int(w).bit_length() for w in words),
                               "P": [hex(v) for v in c.P], "S0_first4": [hex(c.S[0][i]) for i in range(4)],
                               "S3_last4": [hex(c.S[3][i]) for i in range(252, 256)]})
    c = oracle.bf_init(workload.CFG4_KEY)
    words = workload.gen_words(workload.SEEDS[4], 2048)
    ct = oracle.bf_ecb(c, words.copy())
    bf["cfg4"] = {"key": workload.CFG4_KEY.hex(), "seed": workload.SEEDS[4], "pairs": 1024,
                  "plain_sha256": hashlib.sha256(words.tobytes()).hexdigest(),
                  "cipher_sha256": hashlib.sha256(ct.tobytes()).hexdigest(),
                  "cipher_first8": [hex(int(v)) for v in ct[:16]]}
    check_blowfish64(bf)     # second derivation: every word reproduced by the big-integer restatement
    bf["second_derivation"] = ("tests/golden/make_golden.py BigIntBlowfish: Python big integers mod 2^64, pi by "
                               "Chudnovsky; reproduces every context and cipher word above")
    dump("blowfish64.json", bf)

    msg = bytearray(workload.gen_records(seed, 3, 1, 200).tobytes())
    before = bytes(msg)
    ctx = oracle.Sha1Ctx()
    oracle.lib().orc_sha1_init(ctypes.byref(ctx))
    cbuf = (ctypes.c_uint8 * len(msg)).from_buffer(msg)
    oracle.lib().orc_sha1_update(ctypes.byref(ctx), cbuf, len(msg))
    dig = ctypes.create_string_buffer(20)
    oracle.lib().orc_sha1_final(ctypes.byref(ctx), dig)
    mb = []
    for size, off, seed_ in ((0, 0, 0x4FD9), (5, 0, 0x4FD9), (100, 0, 0x4FD9), (100, 8, 7), (1023, 3, 12345)):
        # MemBuffer of `size` bytes; the reference grows it and zero-fills before the ECB pass
        # (MemBufferCheckForGrow, mem_buf.c:1525,1934-1992), so room is zero-padded here
        raw = workload.gen_records(seed, 11, 1, size).tobytes() if size else b""
        need = off + 8 * ((size + off) // 8 + 4)
        buf = bytearray(raw) + bytearray(max(0, need - size))
        enc = bytearray(buf)
        new_size = oracle.membuf_encrypt(enc, size, seed_, off)
        dec = bytearray(enc)
        dec_size = oracle.membuf_decrypt(dec, new_size, seed_, off)
        mb.append({"size": size, "offset": off, "seed": seed_, "plain": bytes(buf).hex(),
                   "enc_size": int(new_size), "enc": bytes(enc).hex(), "dec_size": int(dec_size), "dec": bytes(dec).hex()})
    quirks = {
        "source": "oracle",
        "sha1_inplace": {"input": before.hex(), "after_update": bytes(msg).hex(), "digest": dig.raw.hex(),
                         "hashlib_digest": hashlib.sha1(before).hexdigest()},
        "membuffer": mb,
        "membuf_key_4fd9": oracle.membuf_key(0x4FD9).hex(),
    }
    check_quirks(quirks)     # second derivation: ByteArraySha1 and membuffer_crypt reproduce every byte
    quirks["second_derivation"] = ("tests/golden/make_golden.py ByteArraySha1 (sha1.c on a Python bytearray) and "
                                   "membuffer_crypt (mem_buf.c:1499-1617 on BigIntBlowfish) reproduce every byte above")
    dump("quirks.json", quirks)
    # ---- RC4 and the RC4+MD5 frame ----
    for k, p_, c in RC4_KAT:
        key, pt = bytes.fromhex(k), bytes.fromhex(p_)
        assert libcrypto_rc4(key, pt).hex() == c, k
        assert oracle.rc4_crypt(oracle.rc4_init(key), pt)[1].hex() == c, k
    streams = []
    for key, lens in ((b"cryptokey", (1, 2, 3, 64, 1000)), (bytes(range(1, 41)), (300, 5)), (b"\xff", (777,))):
        st = oracle.rc4_init(key)
        data = workload.gen_records(seed, 21, 1, sum(lens)).tobytes()
        outs, pos = [], 0
        for n in lens:            # the state carries across calls (one connection, several buffers)
            st, o = oracle.rc4_crypt(st, data[pos:pos + n])
            outs.append(o.hex())
            pos += n
        assert b"".join(bytes.fromhex(o) for o in outs) == libcrypto_rc4(key, data)
        streams.append({"key": key.hex(), "lens": list(lens), "data": data.hex(), "out": outs, "state_after": st.hex()})
    frames = []
    for i, n in enumerate((0, 1, 2, 3, 26, 55, 56, 63, 64, 65, 100, 1500)):
        key = b"cryptokey" if i % 2 == 0 else bytes([i + 1] * (i + 3))
        st0 = oracle.rc4_init(key)
        payload = workload.gen_records(seed, 40 + i, 1, n).tobytes() if n else b""
        salt = (0x9E3779B9 * (i + 1)) & 0xFFFFFFFF      # arc4random(): upper 4 bytes zero on LP64
        st_w, fr = oracle.rc4md5_frame(st0, payload, salt)
        assert fr == libcrypto_rc4(key, salt.to_bytes(8, "little") + b"HASH:" + hashlib.md5(payload).digest() + b"\0" + payload)
        st_r, dec, ok = oracle.rc4md5_open(st0, fr)
        assert ok == 1 and dec[30:] == payload and st_r == st_w
        frames.append({"key": key.hex(), "salt": salt, "payload": payload.hex(), "frame": fr.hex(),
                       "state_after": st_w.hex()})
    dump("rc4.json", {
        "source": "published KATs (RFC 6229, classic vectors) and oracle frames, all re-checked against "
                  "OpenSSL RC4 + hashlib MD5",
        "kat": [{"key": k, "plain": p_, "cipher": c} for k, p_, c in RC4_KAT],
        "streams": streams,
        "frames": frames,
    })
    print("wrote", sorted(f for f in os.listdir(OUT) if f.endswith(".json")))


if __name__ == "__main__":
    main()
