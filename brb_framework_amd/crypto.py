"""ctypes binding of libbrb_crypto_gpu.so (include/brb_crypto.h).  Test/bench plumbing only."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# BRB_CRYPTO_LIB: another build of the same library for the test plumbing (the ASan/UBSan build of
# tools/sanitize_check.sh); the C library itself reads no environment variable.
LIB_PATH = os.environ.get("BRB_CRYPTO_LIB") or os.path.join(HERE, "libbrb_crypto_gpu.so")
HEADER_PATH = os.path.join(os.path.dirname(HERE), "include", "brb_crypto.h")

BATCH_HOST = 0x0
BATCH_DEVICE = 0x1
BATCH_ASYNC = 0x2
BATCH_ALL_DEVICES = 0x4
BATCH_DROPPED = -2
BATCH_PARTIAL = -3
BATCH_FAULT = -4
TRANSFORM_DROPPED = -1

u8p = ctypes.POINTER(ctypes.c_uint8)
ulp = ctypes.POINTER(ctypes.c_ulong)


class BRB_MD5_CTX(ctypes.Structure):
    """libbrb_data.h:854-860"""
    _fields_ = [("buf", ctypes.c_uint32 * 4), ("bytes", ctypes.c_uint32 * 2), ("in_", ctypes.c_uint32 * 16),
                ("digest", ctypes.c_ubyte * 16), ("string", ctypes.c_ubyte * 64)]


class BrbSha1Ctx(ctypes.Structure):
    """libbrb_data.h:1937-1943"""
    _fields_ = [("state", ctypes.c_uint32 * 5), ("count", ctypes.c_uint32 * 2), ("buffer", ctypes.c_uint8 * 64)]


class BRB_BLOWFISH_CTX(ctypes.Structure):
    """libbrb_data.h:876-879 (LP64: unsigned long = 8 bytes)"""
    _fields_ = [("P", ctypes.c_ulong * 18), ("S", (ctypes.c_ulong * 256) * 4)]


class _Rc4Flags(ctypes.Structure):
    _fields_ = [("initialized", ctypes.c_uint, 1)]


class BRB_RC4_State(ctypes.Structure):
    """libbrb_data.h:887-897"""
    _fields_ = [("perm", ctypes.c_ubyte * 256), ("index1", ctypes.c_ubyte), ("index2", ctypes.c_ubyte),
                ("flags", _Rc4Flags)]


assert ctypes.sizeof(BRB_MD5_CTX) == 168 and ctypes.sizeof(BrbSha1Ctx) == 92
assert ctypes.sizeof(BRB_BLOWFISH_CTX) == 8336 and ctypes.sizeof(BRB_RC4_State) == 264
RC4_STATE_BYTES = 264
RC4MD5_HEADER = 30

_LIB = None

# (name, restype, argtypes) of every function include/brb_crypto.h declares
_SIGNATURES = [
    ("BRB_MD5Init", None, [ctypes.POINTER(BRB_MD5_CTX)]),
    ("BRB_MD5UpdateBig", None, [ctypes.POINTER(BRB_MD5_CTX), ctypes.c_void_p, ctypes.c_ulong]),
    ("BRB_MD5Update", None, [ctypes.POINTER(BRB_MD5_CTX), ctypes.c_void_p, ctypes.c_ulong]),
    ("BRB_MD5UpdateLowerText", None, [ctypes.POINTER(BRB_MD5_CTX), ctypes.c_char_p, ctypes.c_int]),
    ("BRB_MD5Final", None, [ctypes.POINTER(BRB_MD5_CTX)]),
    ("BRB_MD5Transform", None, [ctypes.POINTER(BRB_MD5_CTX)]),
    ("BRB_MD5LateInitDigestString", None, [ctypes.POINTER(BRB_MD5_CTX)]),
    ("BRB_MD5ToStr", None, [ctypes.c_void_p, ctypes.c_void_p]),
    ("BrbSha1_Init", None, [ctypes.POINTER(BrbSha1Ctx)]),
    ("BrbSha1_Update", None, [ctypes.POINTER(BrbSha1Ctx), ctypes.c_void_p, ctypes.c_size_t]),
    ("BrbSha1_Final", None, [ctypes.POINTER(BrbSha1Ctx), ctypes.c_void_p]),
    ("BrbSha1_Transform", None, [ctypes.c_void_p, ctypes.c_void_p]),
    ("BrbSha1_Do", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    ("BRB_Blowfish_Init", None, [ctypes.POINTER(BRB_BLOWFISH_CTX), ctypes.c_void_p, ctypes.c_int]),
    ("BRB_Blowfish_Encrypt", None, [ctypes.POINTER(BRB_BLOWFISH_CTX), ulp, ulp]),
    ("BRB_Blowfish_Decrypt", None, [ctypes.POINTER(BRB_BLOWFISH_CTX), ulp, ulp]),
    ("BRB_RC4_Init", None, [ctypes.POINTER(BRB_RC4_State), ctypes.c_void_p, ctypes.c_int]),
    ("BRB_RC4_Crypt", None, [ctypes.POINTER(BRB_RC4_State), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    ("BRB_MD5BatchFixed", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]),
    ("BRB_MD5Batch", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint,
      ctypes.c_void_p]),
    ("BRB_MD5BatchSegments", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
      ctypes.c_uint, ctypes.c_void_p]),
    ("BRB_MetaDataUnpackBatch", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint,
      ctypes.c_void_p]),
    ("BrbSha1_BatchFixed", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]),
    ("BrbSha1_Batch", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint,
      ctypes.c_void_p]),
    ("BRB_Blowfish_EncryptBatch", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint, ctypes.c_void_p]),
    ("BRB_Blowfish_DecryptBatch", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint, ctypes.c_void_p]),
    ("BRB_RC4_CryptBatch", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
      ctypes.c_uint, ctypes.c_void_p]),
    ("BRB_RC4MD5_FrameBatch", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
      ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint, ctypes.c_void_p]),
    ("BRB_RC4MD5_OpenBatch", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
      ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]),
    ("BRB_Base64EncodeBatch", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
      ctypes.c_uint, ctypes.c_void_p]),
    ("BRB_Base64DecodeBatch", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
      ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]),
    ("BRB_MemBufferKey", None, [ctypes.c_uint, ctypes.c_void_p]),
    ("BRB_MemBufferEncrypt", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_uint, ctypes.c_ulong, ctypes.POINTER(ctypes.c_ulong), ctypes.c_uint,
      ctypes.c_void_p]),
    ("BRB_MemBufferDecrypt", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_uint, ctypes.c_ulong, ctypes.POINTER(ctypes.c_ulong), ctypes.c_uint,
      ctypes.c_void_p]),
    ("BRB_TransformBatcherCreate", ctypes.c_void_p, [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int]),
    ("BRB_TransformBatcherDestroy", None, [ctypes.c_void_p]),
    ("BRB_TransformBatcherEnable", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int]),
    ("BRB_TransformBatcherRead", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32]),
    ("BRB_TransformBatcherWrite", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64]),
    ("BRB_TransformBatcherFlush", ctypes.c_int64, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("BRB_TransformBatcherFlushAsync", ctypes.c_int64, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("BRB_TransformBatcherGetState", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(BRB_RC4_State)]),
    ("BRB_TransformBatcherInjectFault", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("BRB_CryptoGPU_TestOption", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    ("BRB_CryptoGPU_HostRegister", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]),
    ("BRB_CryptoGPU_HostUnregister", ctypes.c_int, [ctypes.c_void_p]),
    ("BRB_CryptoGPU_Available", ctypes.c_int, []),
    ("BRB_CryptoGPU_DeviceCount", ctypes.c_int, []),
    ("BRB_CryptoGPU_SetDevice", ctypes.c_int, [ctypes.c_int]),
    ("BRB_CryptoGPU_GetDevice", ctypes.c_int, []),
    ("BRB_CryptoGPU_ThreadCleanup", None, []),
    ("BRB_CryptoGPU_LastError", ctypes.c_char_p, []),
    ("BRB_CryptoGPU_AsyncFaultCheck", ctypes.c_int, []),
    ("BRB_CryptoGPU_Version", ctypes.c_char_p, []),
]


def lib() -> ctypes.CDLL:
    """Load the in-tree library; raise if it has not been built (no silent fallback)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `make -C {HERE}` "
                               "(or __graft_entry__.build())")
        # One HIP runtime per process: the PyTorch wheel bundles its own libamdhip64.so.7 and
        # libhsa-runtime64.so.1.  Loading torch first lets the dynamic loader resolve this
        # library's DT_NEEDED libamdhip64.so.7 to that same copy (glibc matches by SONAME);
        # the other order maps two HSA runtimes and the second sees no device.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in _SIGNATURES:
            f = getattr(L, name, None)
            if f is None:
                # An older build (interleaved A/B runs load one): the library still loads, but the
                # first call of a symbol it lacks raises here, naming it, instead of failing later
                # with default ctypes argtypes.  tests/test_abi.py checks exports == header.
                setattr(L, name, _missing_symbol(name))
                continue
            f.restype = res
            f.argtypes = args
        _LIB = L
    return _LIB


def _missing_symbol(name: str):
    def call(*_a, **_k):
        raise RuntimeError(f"{LIB_PATH} does not export {name} (a stale build?): rebuild with `make -C {HERE}`")
    return call


def exported_symbols() -> set:
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], check=True, capture_output=True, text=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if ln.strip()}


def gpu_available() -> bool:
    return bool(lib().BRB_CryptoGPU_Available())


def async_fault_check() -> None:
    """BRB_CryptoGPU_AsyncFaultCheck: raises (returned -4) if a wave-pair kernel of this thread's
    async device-mode calls reported a protocol fault since the last check.  Synchronise first."""
    _check(lib().BRB_CryptoGPU_AsyncFaultCheck(), "BRB_CryptoGPU_AsyncFaultCheck")


def test_option(name: str, value: int) -> int:
    """BRB_CryptoGPU_TestOption: sets a process-wide A/B switch, returns its previous value."""
    old = ctypes.c_int(0)
    _check(lib().BRB_CryptoGPU_TestOption(name.encode(), int(value), ctypes.byref(old)), "BRB_CryptoGPU_TestOption")
    return old.value


class TestOption:
    """Context manager: `with TestOption("var_line", 0): ...` restores the previous value on exit."""

    __test__ = False     # not a pytest class

    def __init__(self, name: str, value: int):
        self.name, self.value, self.old = name, value, None

    def __enter__(self):
        self.old = test_option(self.name, self.value)
        return self

    def __exit__(self, *exc):
        test_option(self.name, self.old)
        return False


def _check(rc: int, what: str) -> None:
    if rc != 1:
        msg = lib().BRB_CryptoGPU_LastError().decode(errors="replace")
        raise RuntimeError(f"{what} returned {rc}: {msg}")


# ---- buffer helpers ---------------------------------------------------------------------------
def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


def _ptr(x) -> int:
    if x is None:
        return 0
    if _is_torch(x):
        return x.data_ptr()
    if isinstance(x, np.ndarray):
        if not x.flags["C_CONTIGUOUS"]:
            raise ValueError("array must be C-contiguous")
        return x.ctypes.data
    raise TypeError(f"unsupported buffer type {type(x)}")


def _mode(data, stream, async_, all_devices=False):
    """(flags, stream_handle) for a buffer: torch CUDA tensor -> device mode, numpy -> host mode
    (all_devices: BRB_BATCH_ALL_DEVICES, host mode only)."""
    if all_devices:
        if _is_torch(data):
            raise ValueError("all_devices needs host (numpy) buffers")
        return BATCH_HOST | BATCH_ALL_DEVICES, 0
    if _is_torch(data):
        if not data.is_cuda:
            raise ValueError("torch tensors must live on a CUDA (HIP) device; pass numpy for host mode")
        import torch
        if stream is None:
            stream = torch.cuda.current_stream(data.device)
        handle = stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)
        return BATCH_DEVICE | (BATCH_ASYNC if async_ else 0), handle
    return BATCH_HOST, (int(stream) if stream is not None else 0)


def _out_like(data, n, width):
    if _is_torch(data):
        import torch
        return torch.empty((n, width), dtype=torch.uint8, device=data.device)
    return np.empty((n, width), dtype=np.uint8)


def _nbytes(x) -> int:
    return x.numel() * x.element_size() if _is_torch(x) else x.nbytes


def _digest_fixed(fn, width, data, rec_len, n, out, stream, async_, all_devices=False):
    if n is None:
        n = _nbytes(data) // rec_len if rec_len else 0
    if rec_len * n > _nbytes(data):
        raise ValueError("data is smaller than rec_len * n")
    if out is None:
        out = _out_like(data, n, width)
    flags, h = _mode(data, stream, async_, all_devices)
    _check(fn(_ptr(data), rec_len, n, _ptr(out), flags, h), fn.__name__)
    return out


def _digest_var(fn, width, data, offsets, lengths, out, stream, async_, all_devices=False):
    n = len(offsets)
    if out is None:
        out = _out_like(data, n, width)
    flags, h = _mode(data, stream, async_, all_devices)
    _check(fn(_ptr(data), _ptr(offsets), _ptr(lengths), n, _ptr(out), flags, h), fn.__name__)
    return out


def md5_batch_fixed(data, rec_len, n=None, out=None, stream=None, async_=False, all_devices=False):
    """BRB_MD5BatchFixed: digests (n, 16) of n records of rec_len bytes stored back to back."""
    return _digest_fixed(lib().BRB_MD5BatchFixed, 16, data, rec_len, n, out, stream, async_, all_devices)


def sha1_batch_fixed(data, rec_len, n=None, out=None, stream=None, async_=False, all_devices=False):
    """BrbSha1_BatchFixed: digests (n, 20)."""
    return _digest_fixed(lib().BrbSha1_BatchFixed, 20, data, rec_len, n, out, stream, async_, all_devices)


def md5_batch(data, offsets, lengths, out=None, stream=None, async_=False, all_devices=False):
    """BRB_MD5Batch: offsets uint64[n], lengths uint32[n] (same memory kind as data)."""
    return _digest_var(lib().BRB_MD5Batch, 16, data, offsets, lengths, out, stream, async_, all_devices)


def md5_batch_segments(data, seg_offsets, seg_lengths, rec_first_seg, out=None, stream=None, async_=False,
                       all_devices=False):
    """BRB_MD5BatchSegments: record i = concatenation of segments rec_first_seg[i] .. rec_first_seg[i+1]-1
    (the MetaData pack digest).  rec_first_seg has n + 1 entries."""
    n = len(rec_first_seg) - 1
    if out is None:
        out = _out_like(data, n, 16)
    flags, h = _mode(data, stream, async_, all_devices)
    _check(lib().BRB_MD5BatchSegments(_ptr(data), _ptr(seg_offsets), _ptr(seg_lengths), _ptr(rec_first_seg), n,
                                      _ptr(out), flags, h), "BRB_MD5BatchSegments")
    return out


# BRB_MetaDataUnpackInfo (include/brb_crypto.h), one per pack
METADATA_INFO_DTYPE = np.dtype([("error_code", "<i4"), ("item_count", "<u4"), ("cur_offset", "<u8"),
                                ("cur_remaining", "<u8"), ("cur_needed", "<u8")])


def metadata_unpack_batch(data, offsets, lengths, out=None, stream=None, async_=False, all_devices=False):
    """BRB_MetaDataUnpackBatch: MetaDataUnpack (meta_data.c:145-328) of pack i = data[offsets[i] ..
    + lengths[i]); returns one BRB_MetaDataUnpackInfo per pack (numpy structured array in host mode,
    an (n, 32) uint8 tensor in device mode)."""
    n = len(offsets)
    if out is None:
        if _is_torch(data):
            import torch
            out = torch.empty((n, METADATA_INFO_DTYPE.itemsize), dtype=torch.uint8, device=data.device)
        else:
            out = np.empty(n, METADATA_INFO_DTYPE)
    flags, h = _mode(data, stream, async_, all_devices)
    _check(lib().BRB_MetaDataUnpackBatch(_ptr(data), _ptr(offsets), _ptr(lengths), n, _ptr(out), flags, h),
           "BRB_MetaDataUnpackBatch")
    return out


def sha1_batch(data, offsets, lengths, out=None, stream=None, async_=False, all_devices=False):
    return _digest_var(lib().BrbSha1_Batch, 20, data, offsets, lengths, out, stream, async_, all_devices)


# ---- Blowfish ------------------------------------------------------------------------------------
def blowfish_init(key: bytes, key_len: int | None = None) -> BRB_BLOWFISH_CTX:
    ctx = BRB_BLOWFISH_CTX()
    kb = ctypes.create_string_buffer(bytes(key), max(len(key), 1))
    lib().BRB_Blowfish_Init(ctypes.byref(ctx), kb, len(key) if key_len is None else key_len)
    return ctx


def blowfish_ctx_bytes(ctx: BRB_BLOWFISH_CTX) -> bytes:
    return ctypes.string_at(ctypes.addressof(ctx), ctypes.sizeof(ctx))


def _bf(fn, ctx, words, n_blocks, stream, async_, all_devices=False):
    """words: uint64 numpy array (host) or int64/uint64 torch CUDA tensor (device), 2 words per block.
    ctx: BRB_BLOWFISH_CTX (host mode) or, in device mode, a CUDA uint8 tensor holding its 8336 bytes
    (a BRB_BLOWFISH_CTX is uploaded for you)."""
    if n_blocks is None:
        n_blocks = _nbytes(words) // 16
    if 16 * n_blocks > _nbytes(words):
        raise ValueError("words holds fewer than n_blocks (xl, xr) pairs")
    flags, h = _mode(words, stream, async_, all_devices)
    if flags & BATCH_DEVICE:
        if isinstance(ctx, BRB_BLOWFISH_CTX):
            import torch
            ctx = torch.frombuffer(bytearray(blowfish_ctx_bytes(ctx)), dtype=torch.uint8).to(words.device)
        cptr = _ptr(ctx)
    else:
        cptr = ctypes.addressof(ctx)
    _check(fn(cptr, _ptr(words), n_blocks, flags, h), fn.__name__)
    return words


def blowfish_encrypt_batch(ctx, words, n_blocks=None, stream=None, async_=False, all_devices=False):
    return _bf(lib().BRB_Blowfish_EncryptBatch, ctx, words, n_blocks, stream, async_, all_devices)


def blowfish_decrypt_batch(ctx, words, n_blocks=None, stream=None, async_=False, all_devices=False):
    return _bf(lib().BRB_Blowfish_DecryptBatch, ctx, words, n_blocks, stream, async_, all_devices)


def device_count() -> int:
    """BRB_CryptoGPU_DeviceCount (0 without a usable device)."""
    return int(lib().BRB_CryptoGPU_DeviceCount())


# ---- RC4 and the RC4+MD5 frame ---------------------------------------------------
def rc4_init(key: bytes, keylen: int | None = None) -> BRB_RC4_State:
    """BRB_RC4_Init into a zeroed state."""
    st = BRB_RC4_State()
    kb = ctypes.create_string_buffer(bytes(key), max(len(key), 1))
    lib().BRB_RC4_Init(ctypes.byref(st), kb, len(key) if keylen is None else keylen)
    return st


def rc4_state_bytes(st: BRB_RC4_State) -> bytes:
    return ctypes.string_at(ctypes.addressof(st), RC4_STATE_BYTES)


def rc4_states(keys) -> np.ndarray:
    """(n, 264) uint8 array of BRB_RC4_Init states, one per key (the batch calls' `states`)."""
    out = np.empty((len(keys), RC4_STATE_BYTES), np.uint8)
    for i, k in enumerate(keys):
        out[i] = np.frombuffer(rc4_state_bytes(rc4_init(k)), np.uint8)
    return out


def _same_kind(ref, *xs):
    for x in xs:
        if x is not None and _is_torch(x) != _is_torch(ref):
            raise ValueError("all buffers of one batch call must be numpy (host) or all CUDA tensors (device)")


def rc4_crypt_batch(states, data, offsets, lengths, out=None, stream=None, async_=False, all_devices=False):
    """BRB_RC4_CryptBatch: stream i = data[offsets[i]:+lengths[i]] -> out (in place when out is None).
    states: (n, 264) uint8, updated in place."""
    out = data if out is None else out
    _same_kind(data, states, out, offsets, lengths)
    flags, h = _mode(data, stream, async_, all_devices)
    _check(lib().BRB_RC4_CryptBatch(_ptr(states), _ptr(data), _ptr(out), _ptr(offsets), _ptr(lengths), len(offsets),
                                    flags, h), "BRB_RC4_CryptBatch")
    return out


def rc4md5_frame_batch(states, payload, offsets, lengths, salts, frames, frame_offsets, stream=None, async_=False,
                       all_devices=False):
    """BRB_RC4MD5_FrameBatch: frames[frame_offsets[i]:+30+lengths[i]] = RC4(salt|"HASH:"|MD5|NUL|payload)."""
    _same_kind(payload, states, offsets, lengths, salts, frames, frame_offsets)
    flags, h = _mode(payload, stream, async_, all_devices)
    _check(lib().BRB_RC4MD5_FrameBatch(_ptr(states), _ptr(payload), _ptr(offsets), _ptr(lengths), _ptr(salts),
                                       _ptr(frames), _ptr(frame_offsets), len(offsets), flags, h),
           "BRB_RC4MD5_FrameBatch")
    return frames


def rc4md5_open_batch(states, frames, offsets, lengths, out=None, valid=None, stream=None, async_=False,
                      all_devices=False):
    """BRB_RC4MD5_OpenBatch: decrypt frames (in place when out is None); returns (out, valid uint8[n])."""
    out = frames if out is None else out
    n = len(offsets)
    if valid is None:
        valid = _out_like(frames, n, 1).reshape(n)
    _same_kind(frames, states, out, offsets, lengths, valid)
    flags, h = _mode(frames, stream, async_, all_devices)
    _check(lib().BRB_RC4MD5_OpenBatch(_ptr(states), _ptr(frames), _ptr(out), _ptr(offsets), _ptr(lengths), n,
                                      _ptr(valid), flags, h), "BRB_RC4MD5_OpenBatch")
    return out, valid


# ---- MemBuffer Blowfish ------------------------------------------------------------
def membuf_span(data_size: int) -> int:
    """BRB_MEMBUF_SPAN: bytes a call touches after buf + offset; data_size = size + offset to
    encrypt, size - offset to decrypt (mem_buf.c:1503, :1557)."""
    return ((data_size // 8 + 3) // 2) * 16


def membuf_key(seed: int) -> bytes:
    k = (ctypes.c_uint * 16)()
    lib().BRB_MemBufferKey(seed, k)
    return bytes(k)


def _membuf(fn, buf, size, seed, offset, stream, decrypt):
    need = offset + membuf_span(size - offset if decrypt else size + offset)
    if _nbytes(buf) < need:
        raise ValueError(f"buffer holds {_nbytes(buf)} bytes, the call needs {need}")
    flags, h = _mode(buf, stream, False)
    ns = ctypes.c_ulong(0)
    _check(fn(_ptr(buf), size, seed, offset, ctypes.byref(ns), flags, h), fn.__name__)
    return ns.value


def membuf_encrypt(buf, size, seed, offset=0, stream=None):
    """BRB_MemBufferEncrypt in place; returns the new MemBuffer size."""
    return _membuf(lib().BRB_MemBufferEncrypt, buf, size, seed, offset, stream, False)


def membuf_decrypt(buf, size, seed, offset=0, stream=None):
    """BRB_MemBufferDecrypt in place; returns the new MemBuffer size."""
    return _membuf(lib().BRB_MemBufferDecrypt, buf, size, seed, offset, stream, True)


# ---- base64 -------------------------------------------------------------------------
def base64_encode_batch(data, offsets, lengths, out, out_offsets, stream=None, async_=False, all_devices=False):
    """BRB_Base64EncodeBatch: out[out_offsets[i]:+4*ceil(len/3)] = base64 of record i."""
    _same_kind(data, offsets, lengths, out, out_offsets)
    flags, h = _mode(data, stream, async_, all_devices)
    _check(lib().BRB_Base64EncodeBatch(_ptr(data), _ptr(offsets), _ptr(lengths), len(offsets), _ptr(out),
                                       _ptr(out_offsets), flags, h), "BRB_Base64EncodeBatch")
    return out


def base64_decode_batch(text, offsets, lengths, out, out_offsets, out_lengths=None, stream=None, async_=False,
                        all_devices=False):
    """BRB_Base64DecodeBatch: returns out_lengths (uint32[n])."""
    n = len(offsets)
    if out_lengths is None:
        if _is_torch(text):
            import torch
            out_lengths = torch.zeros(n, dtype=torch.int32, device=text.device)
        else:
            out_lengths = np.zeros(n, np.uint32)
    _same_kind(text, offsets, lengths, out, out_offsets, out_lengths)
    flags, h = _mode(text, stream, async_, all_devices)
    _check(lib().BRB_Base64DecodeBatch(_ptr(text), _ptr(offsets), _ptr(lengths), n, _ptr(out), _ptr(out_offsets),
                                       _ptr(out_lengths), flags, h), "BRB_Base64DecodeBatch")
    return out_lengths


# ---- receive-loop batching ---------------------------------------------------------
CRYPTO_FUNC_RC4, CRYPTO_FUNC_RC4_MD5 = 1, 2
BATCHER_ZERO_COPY = 0x100
BATCHER_PIPELINED = 0x200    # BRB_BATCHER_PIPELINED: two arenas, flush_async()
BATCHER_ALL_DEVICES = 0x400  # BRB_BATCHER_ALL_DEVICES: connections partitioned over the devices
OP_READ, OP_WRITE = 0, 1
TransformDone = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32,
                                 ctypes.c_int)


class HostRegion:
    """Page-aligned host memory page-locked for the GPU (BRB_CryptoGPU_HostRegister)."""

    def __init__(self, size: int):
        import mmap
        self._L = lib()
        self.size = size
        self._mm = mmap.mmap(-1, size)
        self._view = (ctypes.c_char * size).from_buffer(self._mm)
        self.addr = ctypes.addressof(self._view)
        _check(self._L.BRB_CryptoGPU_HostRegister(self.addr, size), "BRB_CryptoGPU_HostRegister")

    def close(self):
        if self._mm is not None:
            self._L.BRB_CryptoGPU_HostUnregister(self.addr)
            del self._view
            self._mm.close()
            self._mm = None

    def __del__(self):
        self.close()


class TransformBatcher:
    """BRB_TransformBatcher*: one event-loop round of many connections per GPU call.

    zero_copy=True creates the batcher with BRB_BATCHER_ZERO_COPY: the kernels read each buffer in
    place from page-locked host memory.  This wrapper plays the part of a receive loop whose socket
    buffers are page-locked: it keeps one registered region and places each submitted buffer in it
    (the batcher itself copies nothing).

    pipelined=True creates it with BRB_BATCHER_PIPELINED: flush_async() starts the round and returns
    the previous round's results; flush() drains both.  In zero-copy mode the wrapper then keeps one
    region per arena, since a running round's buffers must stay unchanged until delivered."""

    def __init__(self, max_conns: int, max_round_bytes: int, algo: int = CRYPTO_FUNC_RC4_MD5, zero_copy: bool = False,
                 pipelined: bool = False, all_devices: bool = False):
        self._L = lib()
        n_reg = 2 if pipelined else 1
        self._regions = [HostRegion(max(max_round_bytes, 1)) for _ in range(n_reg)] if zero_copy else None
        self._cur = 0
        self._used = 0
        self.h = self._L.BRB_TransformBatcherCreate(max_conns, max_round_bytes,
                                                    algo | (BATCHER_ZERO_COPY if zero_copy else 0) |
                                                    (BATCHER_PIPELINED if pipelined else 0) |
                                                    (BATCHER_ALL_DEVICES if all_devices else 0))
        if not self.h:
            raise RuntimeError("BRB_TransformBatcherCreate: " + self._L.BRB_CryptoGPU_LastError().decode())

    def close(self):
        if self.h:
            self._L.BRB_TransformBatcherDestroy(self.h)
            self.h = None
        if self._regions is not None:
            for r in self._regions:
                r.close()
            self._regions = None

    def _place(self, data: bytes):
        """Zero-copy mode: the buffer's address inside the registered region (None when full)."""
        n = len(data)
        region = self._regions[self._cur]
        if self._used + n > region.size:
            return None
        a = region.addr + self._used
        ctypes.memmove(a, bytes(data), n)
        self._used += n
        return a

    def __del__(self):
        self.close()

    def enable(self, conn: int, key: bytes):
        _check(self._L.BRB_TransformBatcherEnable(self.h, conn, bytes(key), len(key)), "BRB_TransformBatcherEnable")

    def read(self, conn: int, data: bytes) -> int:
        if self._regions is not None:
            a = self._place(data)
            return 0 if a is None else self._L.BRB_TransformBatcherRead(self.h, conn, a, len(data))
        return self._L.BRB_TransformBatcherRead(self.h, conn, bytes(data), len(data))

    def write(self, conn: int, data: bytes, salt: int) -> int:
        if self._regions is not None:
            a = self._place(data)
            return 0 if a is None else self._L.BRB_TransformBatcherWrite(self.h, conn, a, len(data), salt)
        return self._L.BRB_TransformBatcherWrite(self.h, conn, bytes(data), len(data), salt)

    def _run(self, fn_name):
        res = []

        def cb(_user, conn, op, out, n, valid):
            res.append((conn, op, ctypes.string_at(out, n) if n else b"", valid))

        fn = TransformDone(cb)
        launched = self._used > 0
        rc = getattr(self._L, fn_name)(self.h, fn, None)
        if rc in (BATCH_DROPPED, BATCH_PARTIAL):
            # DROPPED: every buffer came back through its callback, those of the dropped round with
            # valid == TRANSFORM_DROPPED and no output.  PARTIAL: the parts that delivered did; the
            # others' rounds stay pending for the next flush.  Either way the delivered results ride
            # on the exception.
            err = RuntimeError(fn_name + ": " + self._L.BRB_CryptoGPU_LastError().decode())
            err.results = res
            err.code = rc
            if rc == BATCH_DROPPED:
                if fn_name.endswith("Async") and launched and self._regions is not None and len(self._regions) == 2:
                    self._cur ^= 1
                self._used = 0
            raise err
        if rc < 0 or (rc == 0 and self._L.BRB_CryptoGPU_LastError()):
            err = RuntimeError(fn_name + ": " + self._L.BRB_CryptoGPU_LastError().decode())
            err.results = res    # whatever callbacks fired before the failure
            err.code = rc
            raise err
        if fn_name.endswith("Async") and launched and self._regions is not None and len(self._regions) == 2:
            self._cur ^= 1      # the running round keeps its region until delivered
        self._used = 0
        return res

    def flush(self):
        """Returns [(conn, op, out bytes, valid)] in submission order (every round still pending)."""
        return self._run("BRB_TransformBatcherFlush")

    def flush_async(self):
        """Pipelined: starts this round, returns the previous round's [(conn, op, out, valid)]."""
        return self._run("BRB_TransformBatcherFlushAsync")

    def inject_fault(self, launch: int) -> None:
        """Test support: the `launch`-th kernel launch of every round fails (-1: off)."""
        _check(self._L.BRB_TransformBatcherInjectFault(self.h, launch), "BRB_TransformBatcherInjectFault")

    def state(self, conn: int, op: int) -> bytes:
        st = BRB_RC4_State()
        _check(self._L.BRB_TransformBatcherGetState(self.h, conn, op, ctypes.byref(st)), "BRB_TransformBatcherGetState")
        return rc4_state_bytes(st)
