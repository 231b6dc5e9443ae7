#!/usr/bin/env python3
"""Gather the bench lines one tools/gpu_bench_all.sh pass wrote (gpurun_out/<dir>/<name>.json, one
JSON line each) into profiles/<tag>_bench_lines.json, keyed by name.

Usage: python tools/collect_bench_lines.py gpurun_out/r02c_bench r02c
"""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src, tag = sys.argv[1], sys.argv[2]
    lines = {}
    for f in sorted(glob.glob(os.path.join(src, "*.json"))):
        txt = open(f).read().strip().splitlines()
        if txt:
            lines[os.path.basename(f)[:-5]] = json.loads(txt[-1])
    out = os.path.join(ROOT, "profiles", f"{tag}_bench_lines.json")
    with open(out, "w") as fo:
        json.dump(lines, fo, indent=1, sort_keys=True)
        fo.write("\n")
    for k, v in lines.items():
        r = v.get("roofline") or {}
        print(f"{k:10s} {v.get('value')} {v.get('unit')}  frac {r.get('frac')}  us {r.get('launch_us_avg', r.get('step_us_avg'))}")


if __name__ == "__main__":
    main()
