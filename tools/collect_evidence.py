#!/usr/bin/env python3
"""Evidence for every kept bench line: the rocprofv3 kernel-trace mean of EXACTLY the dispatches
inside the line's timed region, and the line's roofline fraction recomputed from it.

tools/gpu_evidence.sh runs each bench line as
    rocprofv3 --kernel-trace --stats -d <dir>/<line> -o run -- python3 bench.py <args> --mark-timed-region
bench.py then enqueues one tiny `at::cuda::spin_kernel` right before and one right after each timed
region (outside its timing), so the dispatches of a region are the ones that start after the first
sentinel ends and end before the second one starts -- whatever ran before (warm-up, other legs)
or after (host-mode chunks of the pcie leg, the cfg5 sub-measurement) is excluded by construction.
(Round 2's collector took "the last K dispatches" of a kernel name, which after the host-mode leg
were 16 MiB chunks: its cfg4 "timed region" means were not the timed dispatches.)

For each line: per region, the kernels inside it (name, count, mean/min/max duration); the region
whose dispatch count equals the line's steps x kernels per step is the line's timed region; then
    frac_rocprof = bytes_per_step / (sum over the step's kernels of their mean duration) / 8 TB/s
beside the line's own frac (HIP events around the region, which include the ~1-2 us dependent-launch
gap between back-to-back kernels).  Writes <out>/<line>_timed_region.json, copies the --stats kernel
summary, and <out>/lines.json with every line + its check (gpu_evidence.sh runs it on the GPU box,
into gpurun_out/<tag>/evidence; copy that directory to profiles/<tag>_evidence).

Under the profiler every dispatch gets ~1.8 us of extra gap (cfg2: 22.74 us per step by the
events of the profiled run, 20.89 us rocprof kernel mean, 20.99 us by the events of an unprofiled
run), so the line to compare with the rocprof mean is the UNPROFILED one: with a third argument
(the directory of tools/gpu_bench_all.sh's unprofiled lines, same names) each entry also carries
that line's frac and its ratio to frac_rocprof.

Usage: python3 tools/collect_evidence.py gpurun_out/<tag> <out dir> [gpurun_out/<unprofiled tag>]
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import kernel_id  # noqa: E402  (stdlib-only at import)
PEAK = 8000.0
SENTINEL = "spin_kernel"


def dispatches(trace_csv):
    rows = []
    with open(trace_csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def regions(rows):
    """[(kernel name -> [durations ns], in dispatch order) per region between consecutive sentinel pairs]."""
    sent = [(s, e) for s, e, n in rows if SENTINEL in n]
    out = []
    for i in range(0, len(sent) - 1, 2):
        lo, hi = sent[i][1], sent[i + 1][0]
        acc = {}
        for s, e, n in rows:
            if s >= lo and e <= hi and SENTINEL not in n:
                acc.setdefault(n, []).append(e - s)
        out.append({"span_us": round((hi - lo) / 1e3, 3), "kernels": acc})
    return out


def series(v, buckets=16):
    """Mean duration (us) of consecutive slices of the dispatches, in order: a drift from the first
    slices to the last shows the clock settling under sustained load."""
    n = len(v)
    if n < buckets:
        return None
    return [round(sum(v[b * n // buckets:(b + 1) * n // buckets]) / ((b + 1) * n // buckets - b * n // buckets) / 1e3, 2)
            for b in range(buckets)]


def short(name):
    return name if len(name) <= 160 else name[:157] + "..."


def line_check(line, regs):
    """Pick the timed region of `line` and recompute its fraction."""
    r = line.get("roofline") or {}
    steps = int(line.get("steps", 0))
    bytes_step = r.get("bytes_per_launch") or r.get("bytes_per_step")
    event_us = r.get("launch_us_avg") or r.get("step_us_avg")
    for reg in regs:
        ks = reg["kernels"]
        n = sum(len(v) for v in ks.values())
        if steps and n in (steps, 2 * steps):             # one or two kernels per step
            per_step_us = sum(sum(v) / len(v) * len(v) / steps for v in ks.values()) / 1e3
            out = {"timed_dispatches": n, "kernels_per_step": n // steps, "steps": steps,
                   "kernels": {short(k): {"count": len(v), "mean_us": round(sum(v) / len(v) / 1e3, 3),
                                          "min_us": round(min(v) / 1e3, 3), "max_us": round(max(v) / 1e3, 3),
                                          "series_us": series(v)}
                               for k, v in ks.items()},
                   "rocprof_us_per_step": round(per_step_us, 3), "bench_event_us_per_step": event_us,
                   "region_span_us": reg["span_us"]}
            if bytes_step:
                fr = bytes_step / (per_step_us * 1e-6) / 1e9 / PEAK
                out["bytes_per_step"] = bytes_step
                out["frac_rocprof"] = round(fr, 4)
                out["frac_line"] = r.get("frac")
                if r.get("frac"):
                    out["frac_line_vs_rocprof"] = round(r["frac"] / fr, 4)
            return out
    return None


def main():
    src, dst = sys.argv[1], sys.argv[2]
    plain = sys.argv[3] if len(sys.argv) > 3 else None
    os.makedirs(dst, exist_ok=True)
    summary = {}
    for bj in sorted(glob.glob(os.path.join(src, "*.json"))):
        name = os.path.splitext(os.path.basename(bj))[0]
        try:
            line = json.load(open(bj))
        except (OSError, ValueError):
            continue
        traces = glob.glob(os.path.join(src, name, "**", "run_kernel_trace.csv"), recursive=True)
        stats = glob.glob(os.path.join(src, name, "**", "run_kernel_stats.csv"), recursive=True)
        entry = {"line": line}
        if traces:
            regs = regions(dispatches(traces[0]))
            chk = line_check(line, regs)
            entry["timed_region"] = chk
            comp = (line.get("roofline") or {}).get("compute") or {}
            if chk and comp:
                # the line's compute / traffic must come from a PMC pass of the kernels it timed
                timed = sorted(kernel_id(k) for k in chk["kernels"])
                chk["timed_kernel_ids"] = timed
                chk["compute_kernels"] = comp.get("kernels")
                chk["compute_kernels_match"] = comp.get("kernels") == timed
                if not chk["compute_kernels_match"]:
                    print(f"WARNING {name}: roofline.compute from {comp.get('kernels')} "
                          f"({comp.get('refused') or comp.get('source')}), timed {timed}", file=sys.stderr)
            if "cfg5" in line:
                sub = dict(line["cfg5"])
                sub["roofline"] = {"launch_us_avg": sub.get("launch_us_avg"),
                                   "bytes_per_launch": sub["records_per_gpu"] * 1500,
                                   "frac": sub.get("roofline_frac")}
                entry["cfg5_timed_region"] = line_check(sub, regs)
            with open(os.path.join(dst, f"{name}_timed_region.json"), "w") as f:
                json.dump({k: v for k, v in entry.items() if k != "line"}, f, indent=1)
                f.write("\n")
        if plain and entry.get("timed_region"):
            try:
                pl = json.load(open(os.path.join(plain, name + ".json")))
            except (OSError, ValueError):
                pl = None
            if pl and (pl.get("roofline") or {}).get("frac"):
                t = entry["timed_region"]
                t["frac_unprofiled_line"] = pl["roofline"]["frac"]
                t["unprofiled_event_us_per_step"] = pl["roofline"].get("launch_us_avg", pl["roofline"].get("step_us_avg"))
                if t.get("frac_rocprof"):
                    t["frac_unprofiled_vs_rocprof"] = round(pl["roofline"]["frac"] / t["frac_rocprof"], 4)
                entry["unprofiled_line"] = pl
            with open(os.path.join(dst, f"{name}_timed_region.json"), "w") as f:
                json.dump({k: v for k, v in entry.items() if k not in ("line", "unprofiled_line")}, f, indent=1)
                f.write("\n")
        if stats:
            shutil.copy(stats[0], os.path.join(dst, f"{name}_kernel_stats.csv"))
        summary[name] = entry
    with open(os.path.join(dst, "lines.json"), "w") as f:
        json.dump(summary, f, indent=1)
        f.write("\n")
    for name, e in summary.items():
        t = e.get("timed_region") or {}
        print(f"{name:9s} rocprof {t.get('rocprof_us_per_step')} us -> frac {t.get('frac_rocprof')} | unprofiled line "
              f"{t.get('unprofiled_event_us_per_step')} us frac {t.get('frac_unprofiled_line')} "
              f"(ratio {t.get('frac_unprofiled_vs_rocprof')}) | profiled line frac {t.get('frac_line')}")


if __name__ == "__main__":
    main()
