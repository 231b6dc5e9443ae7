#!/usr/bin/env python3
"""Instruction mix per basic block of one kernel in a gfx950 device assembly file.

    make -C brb_framework_amd asm          # build/*.s
    python3 tools/asm_blocks.py brb_framework_amd/build/md5_kernels.s 'digest_line_kernel.*Md5Alg.*Li8ELb1ELb1ELb1E'

Prints, for every basic block of the first kernel whose symbol matches the regex: the counts of
VALU (v_*), SALU (s_* other than waits/branches/nops), LDS (ds_*), VMEM (buffer_/global_/flat_)
instructions, the v_cndmask count, and the block's branch targets -- the VALU-per-block accounting
DESIGN.md §4.1a cites.  Measurement tooling only; nothing in the library reads it.
"""
import re
import sys
from collections import Counter


def blocks(path, pat):
    rx = re.compile(pat)
    cur = None
    out = []
    in_fn = False
    with open(path) as f:
        for line in f:
            s = line.strip()
            if not in_fn:
                m = re.match(r"^(_Z\S+):", line)
                if m and rx.search(m.group(1)):
                    in_fn = True
                    cur = {"name": "entry", "c": Counter(), "br": []}
                    out.append(cur)
                continue
            if s.startswith(".Lfunc_end") or s.startswith("s_endpgm") and False:
                break
            m = re.match(r"^(\.LBB\d+_\d+):", line)
            if m:
                cur = {"name": m.group(1), "c": Counter(), "br": []}
                out.append(cur)
                continue
            if not s or s.startswith((";", ".", "//")):
                continue
            op = s.split()[0]
            c = cur["c"]
            if op.startswith("v_"):
                c["valu"] += 1
                if op.startswith("v_cndmask"):
                    c["cndmask"] += 1
                if op.startswith("v_readfirstlane") or op.startswith("v_readlane") or op.startswith("v_writelane"):
                    c["xlane"] += 1
            elif op.startswith("ds_"):
                c["lds"] += 1
            elif op.startswith(("buffer_", "global_", "flat_", "scratch_")):
                c["vmem"] += 1
            elif op.startswith("s_cbranch") or op.startswith("s_branch"):
                c["br"] += 1
                cur["br"].append(s.split()[-1])
            elif op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_setprio", "s_sleep")):
                c["wait"] += 1
            elif op.startswith("s_endpgm"):
                c["end"] += 1
                cur["br"].append("END")
            elif op.startswith("s_"):
                c["salu"] += 1
            if op == "s_endpgm":
                pass
    return out


def main():
    path, pat = sys.argv[1], sys.argv[2]
    bl = blocks(path, pat)
    tot = Counter()
    print(f"{'block':<14}{'valu':>6}{'cnd':>5}{'salu':>6}{'lds':>5}{'vmem':>5}  -> targets")
    for b in bl:
        c = b["c"]
        tot.update(c)
        print(f"{b['name']:<14}{c['valu']:>6}{c['cndmask']:>5}{c['salu']:>6}{c['lds']:>5}{c['vmem']:>5}  -> {' '.join(b['br'])}")
    print(f"{'total':<14}{tot['valu']:>6}{tot['cndmask']:>5}{tot['salu']:>6}{tot['lds']:>5}{tot['vmem']:>5}")


if __name__ == "__main__":
    main()
