#!/usr/bin/env python3
"""Copy the rocprofv3 evidence of one GPU pass (tools/gpu_round.sh) into profiles/ and derive
profiles/pmc_traffic.json, the per-launch HBM traffic bench.py reports as roofline.traffic.

Traffic = (FETCH_SIZE * 2 + WRITE_SIZE) * 1024 bytes per dispatch, mean over the profiled
dispatches.  FETCH_SIZE is doubled per MI355X_MICROARCH.md §HBM: on gfx950 it reports half the
bytes of a 16-B-per-lane streaming read, global_load and buffer_load ... lds alike (our staging is
buffer_load_dwordx4 ... lds); WRITE_SIZE is exact for 16-B-per-lane stores (MD5 digests; the
SHA-1 digests are 4-byte stores, WRITE_SIZE taken as reported).

Usage: python tools/collect_profiles.py gpurun_out/r01 r01
"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import kernel_id  # noqa: E402  (stdlib-only at import)


def pmc_means(d, pat):
    acc = {}
    for p in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
        for row in csv.DictReader(open(p)):
            if pat in row["Kernel_Name"]:
                acc.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def pmc_kernels(d, pat):
    """The distinct kernels (bench.kernel_id) the passes profiled under filter `pat`: bench.py uses
    an entry only for a line whose timed region launches exactly these."""
    ks = set()
    for p in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
        for row in csv.DictReader(open(p)):
            if pat in row["Kernel_Name"]:
                ks.add(kernel_id(row["Kernel_Name"]))
    return sorted(ks)


def timed_region(trace_csv, pat, bench_json):
    """SUPERSEDED by tools/collect_evidence.py (round 3): this takes the last K dispatches matching
    `pat`, which after bench.py's host-mode leg are its 16 MiB chunks, not the timed dispatches
    (What's weak 4).  Kept only so round-2 tags can be re-derived the way they were."""
    try:
        b = json.load(open(bench_json))
    except (OSError, ValueError):
        return None
    per_step = 2 if "bf_rep" in pat else 1                     # cfg4: encrypt + decrypt per step
    k = int(b["steps"]) * per_step
    durs = []
    for row in csv.DictReader(open(trace_csv)):
        if pat in row["Kernel_Name"]:
            durs.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]) - int(row["Start_Timestamp"])))
    durs.sort()
    last = [d for _, d in durs[-k:]]
    if not last:
        return None
    r = b.get("roofline", {})
    return {"kernel_filter": pat, "dispatches_total": len(durs), "timed_dispatches": len(last),
            "rocprof_mean_us_timed_region": round(sum(last) / len(last) / 1e3, 3),
            "rocprof_mean_us_all": round(sum(d for _, d in durs) / len(durs) / 1e3, 3),
            "bench_event_us_per_step": r.get("launch_us_avg", r.get("step_us_avg")),
            "note": "bench_event_us_per_step includes the dependent-launch gap between back-to-back kernels"}


COUNTERS = ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_LDS_IDX_ACTIVE", "SQ_LDS_BANK_CONFLICT",
            "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY",
            "GRBM_GUI_ACTIVE", "SQ_WAVES")


def counters(m):
    """Per-dispatch means of the compute counters bench.py's roofline.compute reads (lower-case keys)."""
    return {k.lower(): m[k] for k in COUNTERS if k in m}


def backfill(tag):
    """Adds the compute counters of the kept profiles/<tag>_pmc_<key>.txt summaries to
    pmc_traffic.json (entries whose details predate them)."""
    prof = os.path.join(ROOT, "profiles")
    path = os.path.join(prof, "pmc_traffic.json")
    traffic = json.load(open(path))
    for key in [k for k in traffic if not k.endswith("_detail")]:
        txt = os.path.join(prof, f"{tag}_pmc_{key}.txt")
        if not os.path.exists(txt):
            continue
        m = {}
        for ln in open(txt):
            parts = ln.split()
            if len(parts) == 2 and parts[0].isupper():
                m[parts[0]] = float(parts[1])
        traffic[key + "_detail"].update(counters(m))
    with open(path, "w") as f:
        json.dump(traffic, f, indent=1, sort_keys=True)
        f.write("\n")


def main():
    if sys.argv[1] == "--backfill":
        backfill(sys.argv[2])
        return
    src, tag = sys.argv[1], sys.argv[2]
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    for sub, name, pat, bj in (("prof", "bench_cfg2_md5", "Md5Alg", "bench_prof.json"),
                               ("prof4", "bench_cfg4_blowfish", "bf_rep", "bench4_prof.json")):
        f = os.path.join(src, sub, "run_kernel_stats.csv")
        if os.path.exists(f):
            shutil.copy(f, os.path.join(prof, f"{tag}_{name}_kernel_stats.csv"))
        t = os.path.join(src, sub, "run_kernel_trace.csv")
        if os.path.exists(t):
            tr = timed_region(t, pat, os.path.join(src, bj))
            if tr:
                with open(os.path.join(prof, f"{tag}_{name}_timed_region.json"), "w") as fo:
                    json.dump(tr, fo, indent=1)
                    fo.write("\n")
    try:                                   # entries of passes this run did not repeat stay
        traffic = json.load(open(os.path.join(prof, "pmc_traffic.json")))
    except (OSError, ValueError):
        traffic = {}
    # (pass directory, key, kernel filter, dispatches per bench step)
    for sub, key, pat, per in (("pmc2", "cfg2_md5", "Md5Alg", 1), ("pmc2s", "cfg2_sha1", "Sha1Alg", 1),
                               ("pmc3", "cfg3_md5", "Md5Alg", 1),
                               ("pmc4", "cfg4_blowfish", "bf_rep_kernel", 1),
                               ("pmc_rc4", "f1_rc4", "rc4_crypt_", 1),
                               ("pmc_rc4md5", "f1_rc4md5", "rc4md5_", 2),
                               ("pmc_md", "f4_metadata", "metadata_", 1),
                               ("pmc_seg", "f4_md5seg", "md5_seg_", 1),
                               ("pmc_b64", "f4_base64", "b64_", 2),
                               ("pmc_md5var", "var_md5var", "Md5Alg", 1),
                               ("pmc_sha1var", "var_sha1var", "Sha1Alg", 1),
                               # the cfg5 shard shape (1 Mi x 1500 B per GPU) as the timed batch
                               ("pmc5", "cfg5_md5", "Md5Alg", 1)):
        d = os.path.join(src, sub)
        if not os.path.isdir(d):
            continue
        summ = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), d, pat],
                              capture_output=True, text=True).stdout
        kern = pmc_kernels(d, pat)
        with open(os.path.join(prof, f"{tag}_pmc_{key}.txt"), "w") as f:
            f.write(f"# rocprofv3 --pmc passes (tools/gpu_pmc.sh), kernel filter '{pat}', mean per dispatch\n")
            f.write(f"# kernels: {kern}\n")
            f.write(summ)
        m = pmc_means(d, pat)
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            fetch = m["FETCH_SIZE"] * 2 * 1024 * per
            write = m["WRITE_SIZE"] * 1024 * per
            traffic[key] = int(fetch + write)
            traffic[key + "_detail"] = {"fetch_bytes": int(fetch), "write_bytes": int(write),
                                        "source": f"profiles/{tag}_pmc_{key}.txt", "kernels": kern,
                                        "formula": "(FETCH_SIZE*2 + WRITE_SIZE) * 1024 per dispatch"
                                                   + (f" x {per} dispatches per step" if per > 1 else ""),
                                        **counters(m)}
    with open(os.path.join(prof, "pmc_traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1, sort_keys=True)
        f.write("\n")
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
