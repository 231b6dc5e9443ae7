"""ctypes binding of the CPU oracle (oracle/brb_oracle.c).  TEST INFRASTRUCTURE ONLY.

Allowed users: tests/, __graft_entry__.smoke() (as the checker) and bench.py's cpu_baseline leg.
The product library never imports, links or calls anything in this directory.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BRB_ORACLE_LIB") or os.path.join(HERE, "liboracle.so")   # sanitizer builds

_L = None
u64 = ctypes.c_uint64
vp = ctypes.c_void_p


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib() -> ctypes.CDLL:
    global _L
    if _L is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        sig = {
            "orc_md5_init": (None, [vp]), "orc_md5_update": (None, [vp, vp, ctypes.c_ulong]),
            "orc_md5_update_big": (None, [vp, vp, ctypes.c_ulong]), "orc_md5_final": (None, [vp]),
            "orc_md5": (None, [vp, u64, vp]),
            "orc_sha1_init": (None, [vp]), "orc_sha1_update": (None, [vp, vp, ctypes.c_size_t]),
            "orc_sha1_final": (None, [vp, vp]), "orc_sha1": (None, [vp, u64, vp]),
            "orc_bf_pi_words": (None, [vp]), "orc_md5_consts": (None, [vp, vp, vp, vp]),
            "orc_sha1_consts": (None, [vp, vp]), "orc_bf_init": (None, [vp, vp, ctypes.c_int]),
            "orc_bf_encrypt": (None, [vp, vp, vp]), "orc_bf_decrypt": (None, [vp, vp, vp]),
            "orc_bf_ecb": (None, [vp, vp, u64, ctypes.c_int, ctypes.c_int]),
            "orc_membuf_key": (None, [ctypes.c_uint, vp]),
            "orc_membuf_encrypt": (u64, [vp, u64, ctypes.c_uint, u64]),
            "orc_membuf_decrypt": (u64, [vp, u64, ctypes.c_uint, u64]),
            "orc_md5_batch_fixed": (None, [vp, ctypes.c_uint32, u64, vp, ctypes.c_int]),
            "orc_sha1_batch_fixed": (None, [vp, ctypes.c_uint32, u64, vp, ctypes.c_int]),
            "orc_md5_batch": (None, [vp, vp, vp, u64, vp]),
            "orc_sha1_batch": (None, [vp, vp, vp, u64, vp]),
            "orc_md5_batch_mt": (None, [vp, vp, vp, u64, vp, ctypes.c_int]),
            "orc_sha1_batch_mt": (None, [vp, vp, vp, u64, vp, ctypes.c_int]),
            "orc_rc4_crypt_batch": (None, [vp, vp, vp, vp, u64, ctypes.c_int]),
            "orc_rc4_init": (None, [vp, vp, ctypes.c_int]),
            "orc_rc4_crypt": (None, [vp, vp, vp, ctypes.c_int]),
            "orc_rc4md5_frame": (None, [vp, vp, u64, u64, vp]),
            "orc_rc4md5_open": (ctypes.c_int, [vp, vp, u64]),
            "orc_rc4md5_frame_batch": (None, [vp, vp, vp, vp, vp, vp, vp, u64, ctypes.c_int]),
            "orc_rc4md5_open_batch": (None, [vp, vp, vp, vp, u64, vp, ctypes.c_int]),
            "orc_b64_encode": (u64, [vp, u64, vp]),
            "orc_b64_decode": (u64, [vp, u64, vp]),
            "orc_metadata_pack": (u64, [vp, vp, vp, vp, vp, u64, vp]),
            "orc_metadata_unpack": (ctypes.c_int, [vp, u64, vp]),
            "orc_metadata_unpack_batch": (None, [vp, vp, vp, u64, vp, ctypes.c_int]),
            "orc_splitmix64": (u64, [u64]),
            "orc_gen_records": (None, [u64, u64, u64, ctypes.c_uint32, vp]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _L = L
    return _L


def _p(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


# ---- digests ----------------------------------------------------------------------------------
def md5(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(16)
    lib().orc_md5(data, len(data), out)
    return out.raw


def sha1(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(20)
    lib().orc_sha1(data, len(data), out)
    return out.raw


def md5_batch_fixed(data: np.ndarray, rec_len: int, n: int, threads: int = 1) -> np.ndarray:
    out = np.empty((n, 16), np.uint8)
    lib().orc_md5_batch_fixed(_p(data), rec_len, n, _p(out), threads)
    return out


def sha1_batch_fixed(data: np.ndarray, rec_len: int, n: int, threads: int = 1) -> np.ndarray:
    out = np.empty((n, 20), np.uint8)
    lib().orc_sha1_batch_fixed(_p(data), rec_len, n, _p(out), threads)
    return out


def md5_batch(data: np.ndarray, offsets: np.ndarray, lengths: np.ndarray, threads: int = 1) -> np.ndarray:
    offsets = np.ascontiguousarray(offsets, np.uint64)
    lengths = np.ascontiguousarray(lengths, np.uint32)
    out = np.empty((len(offsets), 16), np.uint8)
    lib().orc_md5_batch_mt(_p(data), _p(offsets), _p(lengths), len(offsets), _p(out), threads)
    return out


def sha1_batch(data: np.ndarray, offsets: np.ndarray, lengths: np.ndarray, threads: int = 1) -> np.ndarray:
    offsets = np.ascontiguousarray(offsets, np.uint64)
    lengths = np.ascontiguousarray(lengths, np.uint32)
    out = np.empty((len(offsets), 20), np.uint8)
    lib().orc_sha1_batch_mt(_p(data), _p(offsets), _p(lengths), len(offsets), _p(out), threads)
    return out


def rc4_crypt_batch(states: np.ndarray, data: np.ndarray, offsets: np.ndarray, lengths: np.ndarray,
                    threads: int = 1) -> None:
    """BRB_RC4_Crypt in place on every stream; states (n, 264) uint8 advanced in place."""
    offsets = np.ascontiguousarray(offsets, np.uint64)
    lengths = np.ascontiguousarray(lengths, np.uint32)
    lib().orc_rc4_crypt_batch(_p(states), _p(data), _p(offsets), _p(lengths), len(offsets), threads)


class Md5Ctx(ctypes.Structure):
    _fields_ = [("buf", ctypes.c_uint32 * 4), ("bytes", ctypes.c_uint32 * 2), ("in_", ctypes.c_uint32 * 16),
                ("digest", ctypes.c_ubyte * 16), ("string", ctypes.c_ubyte * 64)]


class Sha1Ctx(ctypes.Structure):
    _fields_ = [("state", ctypes.c_uint32 * 5), ("count", ctypes.c_uint32 * 2), ("buffer", ctypes.c_uint8 * 64)]


# ---- Blowfish ---------------------------------------------------------------------------------
class BfCtx(ctypes.Structure):
    _fields_ = [("P", ctypes.c_uint64 * 18), ("S", (ctypes.c_uint64 * 256) * 4)]


def bf_pi_words() -> list:
    w = (ctypes.c_uint32 * 1042)()
    lib().orc_bf_pi_words(w)
    return list(w)


def md5_consts() -> dict:
    """The MD5 constants the restatement uses: T, message word and rotation per step, IV."""
    a = [np.zeros(64, np.uint32) for _ in range(3)] + [np.zeros(4, np.uint32)]
    lib().orc_md5_consts(*[_p(x) for x in a])
    return dict(zip(("T", "word", "rot", "iv"), [x.tolist() for x in a]))


def sha1_consts() -> dict:
    """The SHA-1 constants the restatement uses: round constant per step, IV."""
    k, iv = np.zeros(80, np.uint32), np.zeros(5, np.uint32)
    lib().orc_sha1_consts(_p(k), _p(iv))
    return {"k80": k.tolist(), "iv": iv.tolist()}


def bf_init(key: bytes, key_len: int | None = None) -> BfCtx:
    c = BfCtx()
    kb = ctypes.create_string_buffer(bytes(key), max(len(key), 1))
    lib().orc_bf_init(ctypes.byref(c), kb, len(key) if key_len is None else key_len)
    return c


def bf_ctx_bytes(c: BfCtx) -> bytes:
    return ctypes.string_at(ctypes.addressof(c), ctypes.sizeof(c))


def bf_encrypt(c: BfCtx, xl: int, xr: int, decrypt: bool = False):
    L, R = ctypes.c_uint64(xl), ctypes.c_uint64(xr)
    (lib().orc_bf_decrypt if decrypt else lib().orc_bf_encrypt)(ctypes.byref(c), ctypes.byref(L), ctypes.byref(R))
    return L.value, R.value


def bf_ecb(c: BfCtx, words: np.ndarray, decrypt: bool = False, threads: int = 1) -> np.ndarray:
    """In-place ECB over a uint64 array of (xl, xr) pairs; returns it."""
    assert words.dtype == np.uint64
    lib().orc_bf_ecb(ctypes.byref(c), _p(words), words.size // 2, 1 if decrypt else 0, threads)
    return words


def membuf_encrypt(buf: bytearray, size: int, seed: int, offset: int = 0) -> int:
    cbuf = (ctypes.c_uint8 * len(buf)).from_buffer(buf)
    return lib().orc_membuf_encrypt(cbuf, size, seed, offset)


def membuf_decrypt(buf: bytearray, size: int, seed: int, offset: int = 0) -> int:
    cbuf = (ctypes.c_uint8 * len(buf)).from_buffer(buf)
    return lib().orc_membuf_decrypt(cbuf, size, seed, offset)


def membuf_key(seed: int) -> bytes:
    k = (ctypes.c_uint * 16)()
    lib().orc_membuf_key(seed, k)
    return bytes(k)


# ---- RC4 and RC4+MD5 framing ------------------------------------------------------------------
RC4_STATE_BYTES = 264      # sizeof(BRB_RC4_State), libbrb_data.h:887-897
RC4MD5_HDR = 30            # salt(8) "HASH:"(5) md5(16) NUL(1)


def rc4_init(key: bytes, keylen: int | None = None) -> bytes:
    """BRB_RC4_Init (rc4.c:40-62) into a zeroed 264-byte state; returns the state bytes."""
    st = ctypes.create_string_buffer(RC4_STATE_BYTES)
    kb = ctypes.create_string_buffer(bytes(key), max(len(key), 1))
    lib().orc_rc4_init(st, kb, len(key) if keylen is None else keylen)
    return st.raw


def rc4_crypt(state: bytes, data: bytes) -> tuple[bytes, bytes]:
    """BRB_RC4_Crypt (rc4.c:64-87): returns (new state bytes, output bytes)."""
    st = ctypes.create_string_buffer(bytes(state), RC4_STATE_BYTES)
    out = ctypes.create_string_buffer(max(len(data), 1))
    lib().orc_rc4_crypt(st, bytes(data), out, len(data))
    return st.raw, out.raw[: len(data)]


def rc4md5_frame(state: bytes, payload: bytes, salt: int) -> tuple[bytes, bytes]:
    """WRITE side of EvAIOReqTransform_CryptoRaw (ev_kq_aio_transform.c:212-230, :281-283)."""
    st = ctypes.create_string_buffer(bytes(state), RC4_STATE_BYTES)
    fr = ctypes.create_string_buffer(RC4MD5_HDR + len(payload))
    lib().orc_rc4md5_frame(st, bytes(payload), len(payload), salt, fr)
    return st.raw, fr.raw


def rc4md5_open(state: bytes, frame: bytes) -> tuple[bytes, bytes, int]:
    """READ side (:270-279) + DataValidate (:158-184): returns (new state, decrypted frame, valid)."""
    st = ctypes.create_string_buffer(bytes(state), RC4_STATE_BYTES)
    fr = ctypes.create_string_buffer(bytes(frame), max(len(frame), 1))
    ok = lib().orc_rc4md5_open(st, fr, len(frame))
    return st.raw, fr.raw[: len(frame)], ok


def rc4md5_frame_batch(states, payload, offs, lens, salts, frames, foffs, threads=1):
    """n connections at once (numpy arrays; states (n, 264) uint8 updated in place)."""
    lib().orc_rc4md5_frame_batch(_p(states), _p(payload), _p(offs), _p(lens), _p(salts), _p(frames), _p(foffs),
                                 len(offs), threads)


def rc4md5_open_batch(states, frames, offs, lens, valid, threads=1):
    lib().orc_rc4md5_open_batch(_p(states), _p(frames), _p(offs), _p(lens), len(offs), _p(valid), threads)


def b64_encode(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(4 * ((len(data) + 2) // 3) + 1)
    n = lib().orc_b64_encode(bytes(data), len(data), out)
    return out.raw[:n]


def b64_decode(text: bytes) -> bytes:
    out = ctypes.create_string_buffer(3 * (len(text) // 4) + 1)
    n = lib().orc_b64_decode(bytes(text), len(text), out)
    return out.raw[:n]


# ---- generator ---------------------------------------------------------------
class MdInfo(ctypes.Structure):
    _fields_ = [("error_code", ctypes.c_int32), ("item_count", ctypes.c_uint32), ("cur_offset", ctypes.c_uint64),
                ("cur_remaining", ctypes.c_uint64), ("cur_needed", ctypes.c_uint64)]


def metadata_pack(items) -> bytes:
    """MetaDataPack (meta_data.c:104-140): items = [(item_id, item_sub_id, data bytes), ...]."""
    data = b"".join(d for _, _, d in items)
    lens = np.array([len(d) for _, _, d in items], np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64) if len(items) else np.zeros(0, np.uint64)
    ids = np.array([i for i, _, _ in items], np.uint64)
    subs = np.array([s for _, s, _ in items], np.uint64)
    src = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
    out = np.zeros(64 + int(lens.sum()) + 25 * len(items), np.uint8)
    ptr = lambda a: a.ctypes.data if a.size else None
    n = lib().orc_metadata_pack(_p(src), ptr(offs), ptr(lens), ptr(ids), ptr(subs), len(items), _p(out))
    return out[:n].tobytes()


def metadata_unpack(pack: bytes) -> tuple:
    """MetaDataUnpack (meta_data.c:145-328) -> (error_code, item_count, cur_offset, cur_remaining, cur_needed)."""
    b = np.frombuffer(pack, np.uint8) if pack else np.zeros(1, np.uint8)
    info = MdInfo()
    lib().orc_metadata_unpack(_p(b), len(pack), ctypes.byref(info))
    return (info.error_code, info.item_count, info.cur_offset, info.cur_remaining, info.cur_needed)


def metadata_unpack_batch(data: np.ndarray, offsets: np.ndarray, lengths: np.ndarray, threads: int = 1) -> np.ndarray:
    """orc_metadata_unpack over many packs; rows as BRB_MetaDataUnpackInfo (32 bytes each)."""
    info = np.zeros((len(offsets), 32), np.uint8)
    lib().orc_metadata_unpack_batch(_p(data), _p(offsets), _p(lengths), len(offsets), _p(info), threads)
    return info


def gen_records(seed: int, r0: int, n: int, rec_len: int) -> np.ndarray:
    """C restatement of the deterministic byte generator: n records of rec_len bytes."""
    out = np.empty(n * rec_len, np.uint8)
    lib().orc_gen_records(seed, r0, n, rec_len, _p(out))
    return out
