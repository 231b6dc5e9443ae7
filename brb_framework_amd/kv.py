"""Encrypted K/V files: the crypto side of KVWriteToFile / KVReadFromFile
(libbrb_core/data/utils/key_value.c:464-506) on the GPU MemBuffer Blowfish entry points.

A K/V file is the text of __KVAssembleToMemBuffer (key_value.c:229-260: one `key="value"\\n` line,
or `key=value\\n` without quotes, per pair) passed through MemBufferEncryptData(mb, KV_SEED, 0)
(mem_buf.c:1499-1551) and written with its new MemBuffer size (MemBufferWriteToFile,
mem_buf.c:553-591).  Reading decrypts with MemBufferDecryptData(mb, KV_SEED, 0) (mem_buf.c:1553-1617),
whose keyLen is 64 where encrypt's is 4: the reference does not get its own plaintext back, and
neither does this module (bit-exact with the reference, quirk included; tests/test_membuf.py).
Parsing the text (__KVArrayParse) is not on the crypto path and is not reproduced."""
import numpy as np

from . import crypto

KV_SEED = 0x4FD9   # libbrb_data.h:1254


def kv_assemble(pairs, without_quotes: bool = False) -> bytes:
    """__KVAssembleToMemBuffer (key_value.c:229-260); pairs with a None key or value are skipped."""
    out = []
    for k, v in pairs:
        if k is None or v is None:
            continue
        out.append(f"{k}={v}\n" if without_quotes else f'{k}="{v}"\n')
    return "".join(out).encode()


def _mb(data: bytes, span: int) -> np.ndarray:
    b = np.zeros(max(len(data), span) + 16, np.uint8)
    b[: len(data)] = np.frombuffer(data, np.uint8)
    return b


def kv_encrypt(text: bytes, stream=None) -> bytes:
    """The bytes KVWriteToFile(..., encFlag = 1, ...) writes for an assembled text."""
    b = _mb(text, crypto.membuf_span(len(text)))
    n = crypto.membuf_encrypt(b, len(text), KV_SEED, 0, stream)
    return b[:n].tobytes()


def kv_decrypt(data: bytes, stream=None) -> bytes:
    """The MemBuffer contents KVReadFromFile(..., encFlag = 1) parses for a file's bytes."""
    b = _mb(data, crypto.membuf_span(len(data)))
    n = crypto.membuf_decrypt(b, len(data), KV_SEED, 0, stream)
    return b[:n].tobytes()


def kv_write_file(path, pairs, enc: bool = True, without_quotes: bool = False) -> int:
    """KVWriteToFile (key_value.c:464-479).  Returns 1 like the reference."""
    text = kv_assemble(pairs, without_quotes)
    with open(path, "wb") as f:
        f.write(kv_encrypt(text) if enc else text)
    return 1


def kv_read_file(path, enc: bool = True) -> bytes:
    """The buffer KVReadFromFile (key_value.c:481-506) hands to its parser."""
    with open(path, "rb") as f:
        data = f.read()
    return kv_decrypt(data) if enc else data
