#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes written by tools/gpu_pmc.sh (mean per dispatch of one kernel)."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "digest"
acc = collections.defaultdict(list)
dur = []
for p in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
    for row in csv.DictReader(open(p)):
        if pat not in row["Kernel_Name"]:
            continue
        acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
for p in sorted(glob.glob(f"{d}/p*/run_kernel_trace.csv")):
    for r in csv.DictReader(open(p)):
        if pat in r["Kernel_Name"]:
            dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
m = {k: sum(v) / len(v) for k, v in acc.items()}
for k in sorted(m):
    print(f"{k:28s} {m[k]:14.4g}")
if dur:
    dur.sort()
    print(f"{'kernel_us (median, pmc runs)':28s} {dur[len(dur) // 2]:14.2f}")
w = m.get("SQ_WAVES")
if w and "SQ_WAVE_CYCLES" in m:
    print("per wave (x4 cycles): wave_cycles %.0f active %.0f wait_inst %.0f wait_any %.0f  valu/wave %.0f" % (
        m["SQ_WAVE_CYCLES"] / w * 4, m["SQ_ACTIVE_INST_ANY"] / w * 4, m["SQ_WAIT_INST_ANY"] / w * 4,
        m["SQ_WAIT_ANY"] / w * 4, m["SQ_INSTS_VALU"] / w))
if "FETCH_SIZE" in m:
    print("FETCH_SIZE x2 (gfx950 correction) = %.1f MB per dispatch" % (m["FETCH_SIZE"] * 2 / 1024))
