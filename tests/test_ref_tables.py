"""The constant tables of the product and of the oracle against the reference's own source text.

tests/golden/ref_tables.json holds, per table, the word count and the SHA-256 of the words as
tools/ref_tables.py parsed them out of the reference (in the build container, where /root/reference
exists): Blowfish ORIG_P / ORIG_S (blowfish.c:42-310), the 64 MD5 steps' constants, message words
and rotations plus the IV (md5.c:38-47, 179-245), and the SHA-1 round constant of every step plus
the IV (sha1.c:54-58, 99-118, 132-139).  Here the same hashes are recomputed from

  * the product: csrc/common/blowfish_pi.h (BRB_BF_PI_P / BRB_BF_PI_S, generated from pi by
    tools/gen_pi_tables.py), csrc/gpu/md5_device.h and sha1_device.h (the GPU compressions),
    csrc/host/brb_md5.c and brb_sha1.c (the compat surface);
  * the oracle: orc_bf_pi_words (BBP digits of pi), orc_md5_consts (sin-derived T), orc_sha1_consts;

so a deviation of any of them from the reference's text fails here.  This pins the inputs of the
64-bit Blowfish high halves to the reference (the halves themselves stay "parity unpinned": no
reference-run vector exists)."""
import json
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from ref_tables import md5_steps, words_hash  # noqa: E402

GPU = os.path.join(ROOT, "brb_framework_amd", "csrc", "gpu")
HOST = os.path.join(ROOT, "brb_framework_amd", "csrc", "host")
COMMON = os.path.join(ROOT, "brb_framework_amd", "csrc", "common")


@pytest.fixture(scope="module")
def ref():
    with open(os.path.join(ROOT, "tests", "golden", "ref_tables.json")) as f:
        return json.load(f)


def _read(*p):
    with open(os.path.join(*p)) as f:
        return f.read()


def _hex(text):
    return [int(h, 16) for h in re.findall(r"0x([0-9A-Fa-f]+)[uUlL]*", text)]


def _body(src, decl):
    i = src.index(decl)
    return src[src.index("{", i):src.index("};", i)]


def test_blowfish_tables(ref, orc):
    h = _read(COMMON, "blowfish_pi.h")
    p, s = _hex(_body(h, "BRB_BF_PI_P[18]")), _hex(_body(h, "BRB_BF_PI_S[4][256]"))
    assert words_hash(p) == ref["blowfish_orig_p"]
    assert words_hash(s) == ref["blowfish_orig_s"]
    w = orc.bf_pi_words()
    assert words_hash(w[:18]) == ref["blowfish_orig_p"] and words_hash(w[18:]) == ref["blowfish_orig_s"]


def _md5_hashes(steps, iv):
    return {"md5_T": words_hash([t for t, _, _ in steps]), "md5_word_index": words_hash([k for _, k, _ in steps]),
            "md5_rotation": words_hash([r for _, _, r in steps]), "md5_iv": words_hash(iv)}


def _want_md5(ref):
    return {k: ref[k] for k in ("md5_T", "md5_word_index", "md5_rotation", "md5_iv")}


def test_md5_gpu_compression(ref):
    src = _read(GPU, "md5_device.h")
    steps = md5_steps(src[src.index("md5_compress"):], "BRB_MD5_STEP")
    iv = _hex(src[src.index("md5_iv"):].split(";")[0])
    assert len(steps) == 64 and _md5_hashes(steps, iv) == _want_md5(ref)


def test_md5_host_compat(ref):
    src = _read(HOST, "brb_md5.c")
    steps = md5_steps(src, "STEP")
    init = src[src.index("void BRB_MD5Init"):]
    iv = [int(h, 16) for h in re.findall(r"buf\[\d\]\s*=\s*0x([0-9a-fA-F]+)", init)[:4]]
    assert len(steps) == 64 and _md5_hashes(steps, iv) == _want_md5(ref)


def test_md5_oracle(ref, orc):
    c = orc.md5_consts()
    steps = list(zip(c["T"], c["word"], c["rot"]))
    assert _md5_hashes(steps, c["iv"]) == _want_md5(ref)


def test_sha1_gpu_compression(ref):
    src = _read(GPU, "sha1_device.h")
    body = src[src.index("BRB_DEV void sha1_compress"):]
    consts = {m.group(1): int(m.group(2), 16) for m in re.finditer(r"\b(K\d) = 0x([0-9A-Fa-f]+)", body)}
    k80 = []
    # the 80 steps in source order: R5(F, K, i, W) expands to 5 steps, BRB_SHA1_R(F, K, ...) to one
    for m in re.finditer(r"\bR5\(\w+, (K\d), (\d+), \w+\)|BRB_SHA1_R\(\w+, (K\d),", body[body.index("#define WX(i)"):body.index("#undef W0")]):
        if m.group(1):
            k80 += [consts[m.group(1)]] * 5
        else:
            k80.append(consts[m.group(3)])
    iv = _hex(src[src.index("sha1_iv"):].split(";")[0])
    assert len(k80) == 80
    assert words_hash(k80) == ref["sha1_k80"] and words_hash(iv) == ref["sha1_iv"]


def test_sha1_host_compat(ref):
    src = _read(HOST, "brb_sha1.c")
    k80 = [None] * 80
    for m in re.finditer(r"for \(int i = (\d+); i < (\d+); i\+\+\)\s*\{?\s*(?:[^;]*;\s*)?ROUND\(i, [^;]*?(0x[0-9A-Fa-f]+)u", src):
        for i in range(int(m.group(1)), int(m.group(2))):
            k80[i] = int(m.group(3), 16)
    init = src[src.index("void BrbSha1_Init"):]
    iv = [int(h, 16) for h in re.findall(r"state\[\d\] = 0x([0-9A-Fa-f]+)", init)[:5]]
    assert None not in k80
    assert words_hash(k80) == ref["sha1_k80"] and words_hash(iv) == ref["sha1_iv"]


def test_sha1_oracle(ref, orc):
    c = orc.sha1_consts()
    assert words_hash(c["k80"]) == ref["sha1_k80"] and words_hash(c["iv"]) == ref["sha1_iv"]


def test_tables_file_covers_every_table(ref):
    assert set(ref) - {"_source"} == {"blowfish_orig_p", "blowfish_orig_s", "md5_T", "md5_word_index", "md5_rotation",
                                      "md5_iv", "sha1_k80", "sha1_iv"}
    assert ref["blowfish_orig_s"]["words"] == 1024 and ref["sha1_k80"]["words"] == 80
