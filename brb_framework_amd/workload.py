"""Synthetic workloads of BASELINE.json / SURVEY.md §8(d) (test and bench plumbing, not product code).

byte(r, k) = byte (k mod 8), little-endian, of splitmix64(seed ^ (r * 0x9E3779B97F4A7C15) ^ (k >> 3))
splitmix64(x): z = x + 0x9E3779B97F4A7C15; z = (z ^ z >> 30) * 0xBF58476D1CE4E5B9;
               z = (z ^ z >> 27) * 0x94D049BB133111EB; return z ^ z >> 31
The C restatement (oracle/brb_oracle.c orc_gen_records) must agree byte for byte (tested).
"""
from __future__ import annotations

import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)

SEEDS = {1: 0x5EED0001, 2: 0x5EED0002, 3: 0x5EED0003, 4: 0x5EED0004, 5: 0x5EED0005}

# BASELINE.json "configs" (index = config number)
CONFIGS = {
    1: dict(name="cfg1: 1 x 1 MiB MD5 on the CPU (plumbing)", records=1, rec_len=1 << 20, op="md5"),
    2: dict(name="cfg2: 65536 x 1500 B MD5, 1 GPU", records=65536, rec_len=1500, op="md5"),
    3: dict(name="cfg3: 1048576 x 64 B MD5, 1 GPU", records=1 << 20, rec_len=64, op="md5"),
    4: dict(name="cfg4: 65536 x 16 KiB Blowfish enc+dec, 1 GPU", records=65536, rec_len=16384, op="blowfish"),
    5: dict(name="cfg5: 8388608 x 1500 B MD5, 8 GPUs", records=8 << 20, rec_len=1500, op="md5"),
}
CFG4_KEY = b"brb_framework_k4"


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + GOLDEN
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        return z ^ (z >> np.uint64(31))


def gen_records(seed: int, r0: int, n: int, rec_len: int, chunk: int = 1 << 16) -> np.ndarray:
    """n records of rec_len bytes (flat uint8 array), records r0 .. r0 + n - 1."""
    words = (rec_len + 7) // 8
    out = np.empty((n, rec_len), np.uint8)
    k8 = np.arange(words, dtype=np.uint64)[None, :]
    s = np.uint64(seed)
    for c0 in range(0, n, chunk):
        c1 = min(n, c0 + chunk)
        r = np.arange(r0 + c0, r0 + c1, dtype=np.uint64)[:, None]
        with np.errstate(over="ignore"):
            x = s ^ (r * GOLDEN) ^ k8
        z = splitmix64(x)
        out[c0:c1] = z.view(np.uint8).reshape(c1 - c0, words * 8)[:, :rec_len]
    return out.reshape(-1)


def gen_words(seed: int, n_words: int, r0: int = 0) -> np.ndarray:
    """Blowfish plaintext for cfg4: full 64-bit words, word i = splitmix64(seed ^ (i * GOLDEN))."""
    with np.errstate(over="ignore"):
        i = np.arange(r0, r0 + n_words, dtype=np.uint64)
        return splitmix64(np.uint64(seed) ^ (i * GOLDEN))


def shard(n: int, rank: int, world: int) -> tuple:
    """Contiguous record range of `rank`: [rank*n/world, (rank+1)*n/world)."""
    return (n * rank) // world, (n * (rank + 1)) // world


def conn_part(conn: int, parts: int) -> tuple:
    """Part and local connection id of `conn` in an all-devices transform batcher
    (BRB_BATCHER_ALL_DEVICES): connection c lives on part c % G as its connection c // G."""
    return conn % parts, conn // parts
