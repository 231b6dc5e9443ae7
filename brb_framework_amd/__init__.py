"""brb_framework_amd -- MI355X-native libbrb_core/crypto (MD5, SHA-1, 64-bit-word Blowfish, RC4 and
the RC4+MD5 frame of the comm transform, MemBuffer Blowfish, MetaData digests, base64).

The product is the C-ABI shared library ``libbrb_crypto_gpu.so`` built in this directory
(``make -C brb_framework_amd``); its interface is ``include/brb_crypto.h``.  This Python package is
plumbing for tests and benchmarks: it loads that library with ctypes and exposes its entry points
with the reference's names (``BRB_MD5Init`` ... ``BRB_Blowfish_Decrypt``) plus thin helpers for the
batch surface that accept numpy arrays (host mode) or torch CUDA tensors (device mode).

Nothing here computes a digest or a cipher in Python, and nothing falls back to the CPU: if the
library is missing, ``lib()`` raises; if no GPU is usable, the batch helpers raise ``RuntimeError``
with the library's own reason.
"""
from .crypto import (  # noqa: F401
    BATCH_ALL_DEVICES,
    BATCH_DROPPED,
    TRANSFORM_DROPPED,
    TestOption,
    test_option,
    async_fault_check,
    BATCH_ASYNC,
    BATCH_DEVICE,
    BATCH_HOST,
    BRB_BLOWFISH_CTX,
    BRB_MD5_CTX,
    BRB_RC4_State,
    RC4_STATE_BYTES,
    RC4MD5_HEADER,
    BrbSha1Ctx,
    LIB_PATH,
    CRYPTO_FUNC_RC4,
    CRYPTO_FUNC_RC4_MD5,
    OP_READ,
    OP_WRITE,
    TransformBatcher,
    HostRegion,
    BATCHER_ZERO_COPY,
    BATCHER_PIPELINED,
    BATCHER_ALL_DEVICES,
    base64_decode_batch,
    base64_encode_batch,
    blowfish_ctx_bytes,
    blowfish_decrypt_batch,
    blowfish_encrypt_batch,
    blowfish_init,
    device_count,
    exported_symbols,
    gpu_available,
    lib,
    md5_batch,
    md5_batch_fixed,
    md5_batch_segments,
    metadata_unpack_batch,
    METADATA_INFO_DTYPE,
    membuf_decrypt,
    membuf_encrypt,
    membuf_key,
    membuf_span,
    rc4_crypt_batch,
    rc4_init,
    rc4_state_bytes,
    rc4_states,
    rc4md5_frame_batch,
    rc4md5_open_batch,
    sha1_batch,
    sha1_batch_fixed,
)

__all__ = [
    "BATCH_ASYNC", "BATCH_DEVICE", "BATCH_HOST", "BRB_BLOWFISH_CTX", "BRB_MD5_CTX", "BrbSha1Ctx",
    "LIB_PATH", "blowfish_ctx_bytes", "blowfish_decrypt_batch", "blowfish_encrypt_batch",
    "blowfish_init", "exported_symbols", "gpu_available", "lib", "md5_batch", "md5_batch_fixed",
    "sha1_batch", "sha1_batch_fixed", "BRB_RC4_State", "RC4_STATE_BYTES", "RC4MD5_HEADER", "rc4_crypt_batch",
    "rc4_init", "rc4_state_bytes", "rc4_states", "rc4md5_frame_batch", "rc4md5_open_batch", "membuf_decrypt",
    "membuf_encrypt", "membuf_key", "membuf_span", "md5_batch_segments", "metadata_unpack_batch", "METADATA_INFO_DTYPE", "base64_decode_batch",
    "base64_encode_batch", "CRYPTO_FUNC_RC4", "CRYPTO_FUNC_RC4_MD5", "OP_READ", "OP_WRITE", "TransformBatcher",
    "HostRegion", "BATCHER_ZERO_COPY", "BATCHER_PIPELINED", "BATCH_ALL_DEVICES", "device_count",
    "BATCH_DROPPED", "TRANSFORM_DROPPED", "BATCHER_ALL_DEVICES", "TestOption", "test_option", "async_fault_check",
]
