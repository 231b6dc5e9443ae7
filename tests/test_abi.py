"""The drop-in boundary: libbrb_crypto_gpu.so loads, exports exactly include/brb_crypto.h, links
into an unchanged C caller, and the batch surface refuses (never falls back) without a GPU."""
import ctypes
import hashlib
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "brb_crypto.h")
LIBDIR = os.path.dirname(os.environ.get("BRB_CRYPTO_LIB") or os.path.join(ROOT, "brb_framework_amd", "x"))


def header_functions():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = "\n".join(ln for ln in src.splitlines() if not ln.lstrip().startswith("#"))
    return set(re.findall(r"\b((?:BRB|Brb)\w+)\s*\(", src))


def test_header_declares_reference_symbols():
    fns = header_functions()
    reference = {  # libbrb_data.h:862-869, 881-883, 1947-1951
        "BRB_MD5Init", "BRB_MD5UpdateBig", "BRB_MD5Update", "BRB_MD5UpdateLowerText", "BRB_MD5Final",
        "BRB_MD5Transform", "BRB_MD5LateInitDigestString", "BRB_MD5ToStr",
        "BrbSha1_Init", "BrbSha1_Update", "BrbSha1_Final", "BrbSha1_Transform", "BrbSha1_Do",
        "BRB_Blowfish_Init", "BRB_Blowfish_Encrypt", "BRB_Blowfish_Decrypt",
    }
    assert reference <= fns
    assert {"BRB_MD5BatchFixed", "BRB_MD5Batch", "BrbSha1_BatchFixed", "BrbSha1_Batch",
            "BRB_Blowfish_EncryptBatch", "BRB_Blowfish_DecryptBatch"} <= fns


def test_library_exports_exactly_the_header(brb):
    exported = brb.exported_symbols()
    assert header_functions() == exported


def test_struct_layouts_in_c(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(
        '#include <stddef.h>\n#include <stdio.h>\n#include "brb_crypto.h"\n'
        'int main(void){printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(BRB_MD5_CTX), offsetof(BRB_MD5_CTX, in),'
        ' offsetof(BRB_MD5_CTX, string), sizeof(BrbSha1Ctx), sizeof(BRB_BLOWFISH_CTX),'
        ' offsetof(BRB_BLOWFISH_CTX, S)); return 0;}\n')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    assert out == ["168", "24", "104", "92", "8336", "144"]


def build_caller(tmp_path):
    exe = tmp_path / "compat_caller"
    subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c", "compat_caller.c"), "-L", LIBDIR, "-lbrb_crypto_gpu",
                    f"-Wl,-rpath,{LIBDIR}", "-o", str(exe)], check=True)
    return exe


def run_caller(exe):
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    return dict(ln.split(" ", 1) for ln in out.strip().splitlines())


def caller_records():
    x = 0x5EED0002
    out = bytearray(300 * 1500)
    M = (1 << 64) - 1
    for i in range(len(out)):
        x = (x * 6364136223846793005 + 1442695040888963407) & M
        out[i] = x >> 56
    return bytes(out)


def test_unchanged_c_caller_links_and_agrees(brb, tmp_path):
    exe = build_caller(tmp_path)
    res = run_caller(exe)
    recs = caller_records()
    assert res["meta_md5"] == hashlib.md5(recs[:4500]).hexdigest()
    assert res["rec_last_md5"] == hashlib.md5(recs[-1500:]).hexdigest()
    assert res["rec_last_sha1"] == hashlib.sha1(recs[-1500:]).hexdigest()
    assert res["validate"] == "1" and res["bf_roundtrip"] == "1" and res["rc4_roundtrip"] == "1"
    assert res["rc4_kat"] == "bbf316e8d940af0ad3"
    if res["batch_md5_rc"] == "1":          # GPU present: batch == compat
        assert res["batch_md5_eq"] == "1" and res["batch_sha1_eq"] == "1" and res["batch_bf_eq"] == "1"
        assert res["batch_rc4_eq"] == "1"
    else:                                   # no GPU: refused with a reason, no CPU fallback
        assert res["batch_md5_rc"] == "0" and res["batch_reason"].strip()


def test_batch_refuses_without_gpu(brb):
    if brb.gpu_available():
        pytest.skip("a GPU is present; covered by tests/test_gpu_parity.py")
    import numpy as np
    data = np.zeros(64 * 10, np.uint8)
    with pytest.raises(RuntimeError, match="returned 0"):
        brb.md5_batch_fixed(data, 64)
    with pytest.raises(RuntimeError, match="returned 0"):
        brb.sha1_batch(data, np.zeros(2, np.uint64), np.full(2, 8, np.uint32))
    ctx = brb.blowfish_init(b"k")
    with pytest.raises(RuntimeError, match="returned 0"):
        brb.blowfish_encrypt_batch(ctx, np.zeros(4, np.uint64))


def test_batch_bad_args(brb):
    L = brb.lib()
    assert L.BRB_MD5BatchFixed(None, 64, 3, None, 0, None) == -1
    assert L.BRB_MD5Batch(None, None, None, 3, None, 0, None) == -1
    assert L.BRB_Blowfish_EncryptBatch(None, None, 3, 0, None) == -1
    assert L.BRB_MD5BatchFixed(None, 64, 0, None, 0, None) == 1      # empty batch: nothing to do


def test_batch_refuses_oversized_item_counts(brb):
    """One-lane-per-item kernels take fewer than 2^32 items per call: larger counts are refused
    (-1, "split the batch") before any device work, so this runs without a GPU."""
    import ctypes
    L = brb.lib()
    b = ctypes.create_string_buffer(64)
    n = 1 << 33
    assert L.BRB_RC4_CryptBatch(b, b, b, b, b, n, 0, None) == -1
    assert b"split the batch" in L.BRB_CryptoGPU_LastError()
    assert L.BRB_MD5Batch(b, b, b, n, b, 0, None) == -1
    assert L.BRB_RC4MD5_OpenBatch(b, b, b, b, b, n, b, 0, None) == -1
    assert L.BRB_Base64EncodeBatch(b, b, b, n, b, b, 0, None) == -1
    assert L.BRB_MD5BatchFixed(b, 0, n, b, 0, None) == -1
    assert L.BRB_TransformBatcherCreate(1 << 31, 1 << 20, 1) is None
    assert b"max_conns" in L.BRB_CryptoGPU_LastError()


def test_multi_device_runtime_without_gpu(brb):
    """The multi-device runtime (BRB_CryptoGPU_DeviceCount / SetDevice / GetDevice / ThreadCleanup,
    BRB_BATCH_ALL_DEVICES) checks its arguments before any device work, so this runs here."""
    L = brb.lib()
    b = ctypes.create_string_buffer(64 * 16)
    flags = brb.BATCH_DEVICE | brb.BATCH_ALL_DEVICES
    assert L.BRB_MD5BatchFixed(b, 64, 4, b, flags, None) == -1
    assert b"ALL_DEVICES" in L.BRB_CryptoGPU_LastError()
    assert L.BrbSha1_Batch(b, b, b, 4, b, flags, None) == -1
    assert L.BRB_Blowfish_DecryptBatch(b, b, 4, flags, None) == -1
    L.BRB_CryptoGPU_ThreadCleanup()
    if brb.gpu_available():
        assert L.BRB_CryptoGPU_DeviceCount() >= 1
        return
    assert L.BRB_CryptoGPU_DeviceCount() == 0 and L.BRB_CryptoGPU_LastError()
    assert L.BRB_CryptoGPU_SetDevice(0) == 0 and L.BRB_CryptoGPU_GetDevice() == -1
    data = np.zeros(64 * 4, np.uint8)
    with pytest.raises(RuntimeError, match="returned 0"):
        brb.md5_batch_fixed(data, 64, all_devices=True)


def test_test_option_ranges(brb):
    """BRB_CryptoGPU_TestOption refuses unknown names and values out of range (no device needed).
    "devices" stops at 16: an all-devices batcher's submitting threads keep one chunk entry per
    part's round, 16 of them."""
    old = ctypes.c_int(0)
    L = brb.lib()
    assert L.BRB_CryptoGPU_TestOption(b"devices", 17, ctypes.byref(old)) == -1
    assert b"out of" in L.BRB_CryptoGPU_LastError()
    assert L.BRB_CryptoGPU_TestOption(b"no_such_option", 0, None) == -1
    with brb.TestOption("devices", 16):
        pass
    with brb.TestOption("var_sort", 2):
        pass


def test_missing_symbol_raises_by_name(brb, monkeypatch):
    """A stale library that lacks a header symbol still loads (A/B runs of older builds), but a call
    of that symbol raises at once, naming it (no silent default argtypes)."""
    from brb_framework_amd import crypto
    stub = crypto._missing_symbol("BRB_NoSuchCall")
    with pytest.raises(RuntimeError, match="BRB_NoSuchCall"):
        stub(1, 2)


def test_batcher_and_runtime_refusals(brb):
    """The transform batcher's and the runtime's argument / refusal paths, reached without a device
    (and run under ASan + UBSan by tools/sanitize_check.sh): every call with a
    NULL batcher or a bad argument returns -1 or NULL with a reason, and a fault check with no async
    call pending is clean."""
    L = brb.lib()
    b = ctypes.create_string_buffer(64)
    assert L.BRB_TransformBatcherCreate(0, 1 << 20, 1) is None and b"max_conns" in L.BRB_CryptoGPU_LastError()
    assert L.BRB_TransformBatcherCreate(4, 0, 1) is None
    assert L.BRB_TransformBatcherCreate(4, 1 << 20, 7) is None and b"algo" in L.BRB_CryptoGPU_LastError()
    assert L.BRB_TransformBatcherRead(None, 0, b, 8) == -1
    assert L.BRB_TransformBatcherWrite(None, 0, b, 8, 1) == -1
    assert L.BRB_TransformBatcherEnable(None, 0, b"k", 1) == -1
    assert L.BRB_TransformBatcherFlush(None, None, None) == -1
    assert L.BRB_TransformBatcherFlushAsync(None, None, None) == -1
    assert L.BRB_TransformBatcherInjectFault(None, 0) == -1
    st = brb.BRB_RC4_State()
    assert L.BRB_TransformBatcherGetState(None, 0, 0, ctypes.byref(st)) == -1
    L.BRB_TransformBatcherDestroy(None)
    assert L.BRB_CryptoGPU_HostRegister(None, 64) == -1
    assert L.BRB_CryptoGPU_HostUnregister(b) == -1 and b"not registered" in L.BRB_CryptoGPU_LastError()
    assert L.BRB_CryptoGPU_AsyncFaultCheck() == 1
    if not brb.gpu_available():
        assert L.BRB_TransformBatcherCreate(4, 1 << 20, 1) is None and L.BRB_CryptoGPU_LastError()
        assert L.BRB_TransformBatcherCreate(4, 1 << 20, 2 | brb.BATCHER_ALL_DEVICES) is None
        assert L.BRB_MemBufferEncrypt(b, 16, 7, 0, ctypes.byref(ctypes.c_ulong(0)), 0, None) == 0
        assert L.BRB_MetaDataUnpackBatch(b, b, b, 1, b, 0, None) == 0
        assert L.BRB_MD5BatchSegments(b, b, b, b, 1, b, 0, None) == 0
