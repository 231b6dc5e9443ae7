#!/usr/bin/env python3
"""Pins the constant tables of the oracle and the product to the reference's own source text.

Run only in the build container (it reads /root/reference, which never travels to the GPU box):

    python3 tools/ref_tables.py            # writes tests/golden/ref_tables.json

It parses, from the reference's C source (read as text, nothing of it is compiled or copied):
  * Blowfish ORIG_P[18] and ORIG_S[4][256]          libbrb_core/crypto/blowfish.c:42-310
  * the 64 MD5 steps: additive constant T, message-word index and rotation, in step order, and the
    IV                                              libbrb_core/crypto/md5.c:38-47, 179-245
  * the SHA-1 round constant of each of the 80 steps (the R0..R4 macro of each step) and the IV
                                                    libbrb_core/crypto/sha1.c:54-58, 99-118, 132-139
and stores per table only its word count and the SHA-256 of its words as little-endian uint32 --
hashes, not the table text.  tests/test_ref_tables.py (CPU) recomputes the same hashes from the
product's tables (blowfish_pi.h, md5_device.h, sha1_device.h, the host compat C) and from the
oracle, so a deviation of either from the reference's text fails a test.
"""
import hashlib
import json
import os
import re
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/libbrb_core/crypto"
OUT = os.path.join(ROOT, "tests", "golden", "ref_tables.json")


def words_hash(words) -> dict:
    """{"words": n, "sha256": hex} of the words as little-endian uint32."""
    return {"words": len(words), "sha256": hashlib.sha256(b"".join(struct.pack("<I", w & 0xFFFFFFFF) for w in words)).hexdigest()}


def hex_words(text: str) -> list:
    return [int(h, 16) for h in re.findall(r"0x([0-9A-Fa-f]+)[uUlL]*", text)]


def c_array_body(src: str, decl: str) -> str:
    """Text between the `{` after `decl` and the matching `};`."""
    i = src.index(decl)
    j = src.index("{", i)
    depth, k = 0, j
    while True:
        if src[k] == "{":
            depth += 1
        elif src[k] == "}":
            depth -= 1
            if depth == 0:
                return src[j:k + 1]
        k += 1


def md5_steps(src: str, macro: str) -> list:
    """[(T, word index, rotation)] of every `macro(...)` call, in source order.  Handles both the
    reference's MD5STEP(F, w, x, y, z, ctx->in[k] + T, s) and the product's (F, w, x, y, z, m[k], T, s)."""
    out = []
    for m in re.finditer(r"\b" + re.escape(macro) + r"\(([^;]*?)\);", src):
        args = [a.strip() for a in m.group(1).split(",")]
        if not re.search(r"0x[0-9a-fA-F]+", m.group(1)):
            continue                     # the macro's own definition
        if len(args) == 7:               # reference: data + constant in one argument
            k = int(re.search(r"in\[(\d+)\]", args[5]).group(1))
            t = int(re.search(r"0x([0-9a-fA-F]+)", args[5]).group(1), 16)
            s = int(args[6])
        else:                            # product: m[k], T, s
            k = int(re.search(r"\[(\d+)\]", args[5]).group(1))
            t = int(re.search(r"0x([0-9a-fA-F]+)", args[6]).group(1), 16)
            s = int(args[7])
        out.append((t, k, s))
    return out


def md5_tables(steps: list, iv: list) -> dict:
    assert len(steps) == 64, len(steps)
    return {"md5_T": words_hash([t for t, _, _ in steps]), "md5_word_index": words_hash([k for _, k, _ in steps]),
            "md5_rotation": words_hash([s for _, _, s in steps]), "md5_iv": words_hash(iv)}


def reference_tables() -> dict:
    with open(os.path.join(REF, "blowfish.c")) as f:
        bf = f.read()
    p = hex_words(c_array_body(bf, "ORIG_P[16 + 2]"))
    s = hex_words(c_array_body(bf, "ORIG_S[4][256]"))
    assert len(p) == 18 and len(s) == 1024, (len(p), len(s))
    with open(os.path.join(REF, "md5.c")) as f:
        md5 = f.read()
    steps = md5_steps(md5, "MD5STEP")
    init = md5[md5.index("void BRB_MD5Init"):]
    iv = [int(h, 16) for h in re.findall(r"buf\[\d\]\s*=\s*0x([0-9a-fA-F]+)", init)[:4]]
    with open(os.path.join(REF, "sha1.c")) as f:
        sha = f.read()
    kmac = {m.group(1): int(m.group(2), 16) for m in
            re.finditer(r"#define (R[0-4])\(v,w,x,y,z,i\)[^\n]*?\+(0x[0-9A-Fa-f]+)\+rol", sha)}
    seq = re.findall(r"\b(R[0-4])\([a-e],[a-e],[a-e],[a-e],[a-e], ?(\d+)\)", sha)
    assert [int(i) for _, i in seq] == list(range(80)), "sha1.c round calls"
    k80 = [kmac[r] for r, _ in seq]
    siv = [int(h, 16) for h in re.findall(r"state\[\d\] = 0x([0-9A-Fa-f]+)", sha)[:5]]
    out = {"blowfish_orig_p": words_hash(p), "blowfish_orig_s": words_hash(s), **md5_tables(steps, iv),
           "sha1_k80": words_hash(k80), "sha1_iv": words_hash(siv)}
    out["_source"] = {
        "blowfish_orig_p": "libbrb_core/crypto/blowfish.c:42-48 ORIG_P",
        "blowfish_orig_s": "libbrb_core/crypto/blowfish.c:51-310 ORIG_S",
        "md5_T": "libbrb_core/crypto/md5.c:179-245 MD5STEP constants, step order",
        "md5_word_index": "md5.c:179-245 ctx->in[k] of each MD5STEP",
        "md5_rotation": "md5.c:179-245 rotation of each MD5STEP",
        "md5_iv": "md5.c:38-47 BRB_MD5Init",
        "sha1_k80": "libbrb_core/crypto/sha1.c:54-58 R0..R4 constants, per step by the calls at :99-118",
        "sha1_iv": "sha1.c:132-139 BrbSha1_Init",
        "hash": "sha256 of the words as little-endian uint32 (tools/ref_tables.py words_hash)",
    }
    return out


def main():
    if not os.path.isdir(REF):
        sys.exit(f"{REF} not found: this script runs only in the build container")
    t = reference_tables()
    with open(OUT, "w") as f:
        json.dump(t, f, indent=1, sort_keys=True)
        f.write("\n")
    print(f"wrote {OUT}: " + ", ".join(f"{k} ({v['words']} words)" for k, v in sorted(t.items()) if k != "_source"))


if __name__ == "__main__":
    main()
