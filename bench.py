#!/usr/bin/env python3
"""Benchmark of the libbrb_core/crypto hot path on MI355X (BASELINE.json metric).

Default workload (N = 1): BASELINE config 2 -- 65 536 records x 1500 B, MD5 digest of every record
through BRB_MD5BatchFixed (device mode), inputs resident in HBM.  One "step" = one pass of the hot
path over one batch.  With N GPUs every rank digests its own 65 536-record shard of a global
N x 65 536-record batch (record sharding, no collective on the data path): weak scaling.

Honesty rules applied here:
  * each step reads a batch the previous R-1 steps did not touch (R rotation buffers totalling
    >= 640 MB > the 256 MiB Infinity Cache), so the kernel streams from HBM, not from L3;
  * the timed region is K back-to-back steps, each one C-ABI call (ctypes, arguments resolved
    beforehand), between barrier + synchronize on both sides; value is the whole-job rate (all ranks' bytes / max over ranks of the wall time);
  * untimed before it: W warm-up steps, after (with an explicit --warmup) a settle of the same
    launches for >= --settle-s seconds so a short W starts the region at the loaded clock; the
    line reports the settle ("settle") and W ("warmup") as run;
  * roofline.achieved = bytes per launch / (HIP-event time of the timed region on the launch
    stream / K); digests of the last step are spot-checked against hashlib.

Other workloads for DESIGN.md: --config 1 (one 1 MiB buffer through the compat BRB_MD5* calls on
the CPU, no GPU), --config 3 (1 Mi x 64 B MD5), --config 4 (1 GiB Blowfish enc+dec), --op sha1.
Every digest line also carries a "cfg5" object: 1 048 576 x 1500 B records per GPU (exactly
BASELINE cfg5, 8 388 608 records, at --gpus 8).  Run `python bench.py --help`.
"""
from __future__ import annotations

import argparse
import gc
import hashlib
import json
import math
import os
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s (device-resident) + Mrecords/s over 1500B buffers at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md "Chip-level parameters")
TIMING = ("HIP events on the launch stream from the end of step 2 to the end of step K, / (K-2): back-to-back "
          "launches without the first two after the idle synchronize (the wall time behind `value` includes them); "
          "launch_us_avg_all_k / frac_all_k: the same events over all K launches")
L3_BYTES = 256 << 20
SIMDS = 1024                   # 256 CUs x 4 SIMDs
CLOCK_GHZ = 2.1                # shader clock the chip holds with every CU issuing these kernels:
                               # 2.10-2.16 GHz measured in-kernel (s_memtime / s_memrealtime,
                               # profiles/r02d_md5_tput.txt); 2.4 GHz is the maximum, held only with
                               # a few CUs busy (MI355X_MICROARCH.md "DVFS give-back")
VALU_PEAK_CYC = 2.0            # a wave64 VALU instruction occupies a SIMD-32 for 2 cycles (guide, "SIMD")
LONE_WAVE_CYC = {"md5": 4.30, "sha1": 4.32}   # one wave per SIMD: shader cycles per VALU instruction
                                              # of the product's own compression at the measured clock
                                              # (tools/mb/md5_occ.hip, profiles/r03/md5_sha1_occ.txt;
                                              # round 2's 4.85 / 4.54 were a dependent synthetic chain)


def parse():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps K (default: enough for >= 0.3 s of timed GPU work, at least 200)")
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed warm-up steps W (default: as many as fill >= 1 s, so the GPU clock has "
                         "ramped up before the timed region)")
    ap.add_argument("--config", type=int, default=2, choices=[1, 2, 3, 4, 5])
    ap.add_argument("--op", default="md5", choices=["md5", "sha1", "md5var", "sha1var", "rc4", "rc4md5", "batcher",
                                                  "metadata", "md5seg", "base64"],
                    help="rc4 / rc4md5: SURVEY §8 f1 on the cfg2 shape (65 536 connections x 1500 B); "
                         "metadata / base64: f4 on the same shape")
    ap.add_argument("--records-per-gpu", type=int, default=0, help="override the per-GPU record count")
    ap.add_argument("--rec-len", type=int, default=0, help="override the record length of a digest config")
    ap.add_argument("--streams", type=int, default=1, help="HIP streams the timed steps alternate over")
    ap.add_argument("--two-stream", action="store_true", help="also time the steps over 2 streams")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pcie", action="store_true", help="skip the host-inclusive (PCIe) measurement")
    ap.add_argument("--no-cfg5", action="store_true", help="skip the cfg5 (1 Mi records per GPU) sub-measurement")
    ap.add_argument("--settle-s", type=float, default=1.0,
                    help="with an explicit --warmup: seconds of untimed launches before the W steps (0: none; "
                         "the PMC passes use 0 so their traces hold only the W + K dispatches)")
    ap.add_argument("--cpu-seconds", type=float, default=3.0, help="wall-clock budget of the CPU baseline")
    ap.add_argument("--pmc-summary", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="JSON with per-launch HBM bytes measured by rocprofv3 --pmc (optional)")
    ap.add_argument("--frame-stride", type=int, default=0,
                    help="rc4md5: bytes from one frame's start to the next (default 1530 = back to back; 1536 "
                         "puts every frame on a 64-byte sector boundary: the write-amplification experiment)")
    ap.add_argument("--len-dist", default="uniform", choices=["uniform", "bimodal"],
                    help="md5var / sha1var record lengths: U[1000, 2000] (default) or a bimodal diagnostic")
    ap.add_argument("--test-option", action="append", default=[], metavar="NAME=VALUE",
                    help="BRB_CryptoGPU_TestOption before the run (A/B of kernel selections)")
    ap.add_argument("--mark-timed-region", action="store_true",
                    help="enqueue a tiny spin kernel (at::cuda spin_kernel) right before and right after each "
                         "timed region, outside the timing, so a rocprofv3 kernel trace can select exactly the "
                         "timed dispatches (tools/collect_profiles.py)")
    return ap.parse_args()


def relaunch_distributed(args) -> None:
    """`python bench.py --gpus N` outside torchrun: start torchrun as a child (no exec)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(29500 + os.getpid() % 1000), __file__] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def cgroup_cpu_quota():
    """The lease's CPU quota from the cgroup (v2 cpu.max "<quota> <period>" or "max <period>"; v1
    cpu.cfs_quota_us / cpu.cfs_period_us): (cpus or None when unlimited, the raw text)."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            raw = open(path).read().strip()
        except OSError:
            continue
        q, _, per = raw.partition(" ")
        return (None if q == "max" else float(q) / float(per or 100000)), f"{path}: {raw}"
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return (None if q < 0 else q / per), f"cgroup v1 cfs_quota_us {q} cfs_period_us {per}"
    except (OSError, ValueError):
        return None, "no cgroup cpu quota file"


def cpu_threads() -> int:
    """Threads for the CPU baseline: the lease's CPU share.  A finite cgroup quota decides when it
    has one (floor of quota / period); otherwise the share the harness declares in OMP_NUM_THREADS /
    MAX_JOBS (16 per GPU on the box, where the affinity mask shows the whole 256-CPU host); otherwise
    the affinity mask (this container)."""
    aff = len(os.sched_getaffinity(0))
    quota, _ = cgroup_cpu_quota()
    if quota is not None:
        return max(1, min(aff, int(quota)))
    for var in ("OMP_NUM_THREADS", "MAX_JOBS"):
        if os.environ.get(var, "").isdigit():
            return max(1, min(aff, int(os.environ[var])))
    return max(1, aff)


NOTES = {}     # attached to the bench line as "notes": context that is not a measurement


def core_counts(threads: int, single_core_rate: float) -> dict:
    """`cores` = threads actually used, with the evidence for that number: the cgroup quota, the
    affinity mask, nproc and the declared share.  The whole-mask linear extrapolation of the
    single-core rate is NOT part of the baseline: it goes to the line's "notes", labelled."""
    try:
        nproc = int(subprocess.run(["nproc"], capture_output=True, text=True, timeout=10).stdout.strip())
    except (OSError, ValueError, subprocess.SubprocessError):
        nproc = None
    aff = len(os.sched_getaffinity(0))
    quota, quota_raw = cgroup_cpu_quota()
    declared = {v: os.environ[v] for v in ("OMP_NUM_THREADS", "MAX_JOBS") if v in os.environ}
    NOTES["cpu_all_affinity_cpus_extrapolated_gib_s"] = {
        "value": round(single_core_rate * aff, 3),
        "what": f"single-core rate x {aff} affinity CPUs: a linear extrapolation, NOT measured, not the baseline"}
    why = (f"cgroup quota {quota:g} CPUs" if quota is not None else
           f"cgroup quota unlimited ({quota_raw}); the lease's declared share {declared}" if declared else
           f"cgroup quota unlimited ({quota_raw}); the affinity mask")
    return {"cores": threads, "cores_evidence": {"cgroup_cpu_max": quota_raw, "cgroup_quota_cpus": quota,
                                                 "affinity_cpus": aff, "nproc": nproc, "declared_share": declared,
                                                 "threads_used_because": why}}


def kernel_id(name: str) -> str:
    """A rocprofv3 kernel name without `void`, namespaces and the argument list: the kernel and its
    template arguments, e.g. "rc4_crypt_pair_kernel<false>", "digest_line_kernel<Md5Alg, 8, true,
    true>".  tools/collect_profiles.py records these in pmc_traffic.json."""
    n = name.strip()
    if n.startswith("void "):
        n = n[5:]
    n = n.replace("(anonymous namespace)::", "")
    depth = 0
    for i, ch in enumerate(n):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            n = n[:i]
            break
    return re.sub(r"\b[A-Za-z_]\w*::", "", n).strip()


def timed_kernel_patterns(key, opt):
    """Regexes (on kernel_id) of the kernels one step of bench line `key` launches, as the launchers
    in csrc/gpu/*.hip select them under the current test options (`opt(name)` reads one), one regex
    per kernel of the step.  None for a key without PMC evidence."""
    seg = opt("seg_line")
    rc4_pair = opt("rc4_pair") != 0 and opt("rc4_sector") < 0
    table = {
        # <Alg, waves, output 16-aligned, TAIL_HI>: the only forms launch_fixed_line launches
        "cfg2_md5": [r"digest_line_kernel<Md5Alg, 8, (true|false), (true|false)>"],
        "cfg2_sha1": [r"digest_line_kernel<Sha1Alg, 8, (true|false), (true|false)>"],
        "cfg3_md5": [r"digest_b64r_kernel<Md5Alg, .*>"],
        "cfg4_blowfish": [r"bf_rep_kernel<\d+, false>", r"bf_rep_kernel<\d+, true>"],
        "f1_rc4": [r"rc4_crypt_pair_kernel<false>"] if rc4_pair else [r"rc4_crypt_kernel<(true|false)>"],
        "f1_rc4md5": ([r"rc4md5_frame_pair_kernel<false>", r"rc4md5_open_pair_kernel<false>"] if opt("rc4md5_pair")
                      else [r"rc4md5_frame_kernel(<.*>)?", r"rc4md5_open_kernel(<.*>)?"]),
        "f4_metadata": {2: [r"metadata_line_kernel<\d+, \d+, true, false>"],
                        1: [r"metadata_line_kernel<\d+, \d+, false, false>"],
                        0: [r"metadata_unpack_kernel"]}[seg],
        "f4_md5seg": {2: [r"md5_seg_pc_kernel<\d+, false>"], 1: [r"md5_seg_line_kernel<\d+, \d+>"],
                      0: [r"md5_seg_kernel"]}[seg],
        "f4_base64": [r"b64_encode_group_kernel", r"b64_decode_group_kernel"],
        "var_md5var": [r"digest_var_line_kernel<Md5Alg, .*>"] if opt("var_line") else [r"md5_any_kernel<.*>"],
        "var_sha1var": [r"digest_var_line_kernel<Sha1Alg, .*>"] if opt("var_line") else [r"sha1_any_kernel<.*>"],
    }
    return table.get(key)


def kernels_match(pmc_kernels, patterns) -> bool:
    """Every kernel of the PMC pass is one the timed region launches, and every kernel the timed
    region launches was profiled (one to one)."""
    if not pmc_kernels or not patterns or len(pmc_kernels) != len(patterns):
        return False
    left = list(pmc_kernels)
    for p in patterns:
        hit = next((k for k in left if re.fullmatch(p, k)), None)
        if hit is None:
            return False
        left.remove(hit)
    return not left


OPT = None   # set by main(): reads a BRB_CryptoGPU_TestOption value


def load_pmc(path, key, opt=None):
    """(traffic bytes, detail dict, refusal) measured by rocprofv3 --pmc for `key`.  The entry is
    used only if the kernels it profiled ("kernels", kernel_id form) are the ones this line's timed
    region launches (timed_kernel_patterns under the current test options): otherwise (None, None,
    reason) -- a line never carries another kernel's traffic or bound."""
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None, "no PMC summary"
    det = d.get(key + "_detail")
    if det is None:
        return None, None, f"no PMC entry {key}"
    opt = opt or OPT
    pats = timed_kernel_patterns(key, opt) if opt else None
    got = det.get("kernels")
    if pats is None or not kernels_match(got, pats):
        return None, None, (f"PMC entry {key} ({det.get('source')}) profiled {got}, the timed region launches "
                            f"{pats}: not used")
    return d.get(key), det, None


def traffic_fields(path, key, per_step=1):
    t, det, why = load_pmc(path, key)
    if why:
        return {"traffic": None, "traffic_source": why}
    src = det.get("source")
    return {"traffic": t * per_step if t else None,
            "traffic_source": (f"{src}: rocprofv3 --pmc passes of an earlier run (tools/gpu_pmc.sh), not this run; "
                               f"kernels {det.get('kernels')}")}


def compute_fraction(path, key, launch_s, cyc_lone):
    """roofline.compute: the VALU-issue ceiling.  insts = SQ_INSTS_VALU per dispatch (rocprofv3
    --pmc, chip-wide sum of wave-instructions); per SIMD = insts / 1024.  frac_peak = that many
    instructions at the SIMD's peak issue (2 cycles per wave64 instruction) and CLOCK_GHZ over the
    launch time; frac_lone_wave = the same at the cost per instruction measured for the product's
    compression at one wave per SIMD (tools/mb/md5_occ.hip).  That cost is close to the SIMD's
    rate for the mix at any wave count (4.30 / 4.11 / 4.03 cycles at 1 / 2 / 4 waves per SIMD),
    so it is the compute ceiling of cfg3/cfg5 too."""
    _, det, why = load_pmc(path, key)
    if why:
        return {"refused": why}
    if "sq_insts_valu" not in det:
        return None
    per_simd = det["sq_insts_valu"] / SIMDS
    cyc = launch_s * CLOCK_GHZ * 1e9
    out = {"bound": "valu-issue", "sq_insts_valu_per_launch": det["sq_insts_valu"],
           "valu_per_simd": round(per_simd, 1), "clock_ghz": CLOCK_GHZ,
           "peak_cycles_per_inst": VALU_PEAK_CYC, "frac_peak": round(per_simd * VALU_PEAK_CYC / cyc, 4),
           "source": det.get("source"), "kernels": det.get("kernels")}
    if cyc_lone:
        out["lone_wave_cycles_per_inst"] = cyc_lone
        out["frac_lone_wave"] = round(per_simd * cyc_lone / cyc, 4)
        out["note"] = ("frac_lone_wave: VALU per SIMD x the compression's measured cycles per instruction at "
                       "one wave per SIMD (four waves per SIMD run it only ~7% faster) / launch cycles at clock_ghz")
    return out


ISSUE_CYC_LONE = 4.3   # shader cycles per issued instruction of a lone wave (tools/mb/md5_occ.hip, valu_mix.hip)
ISSUE_CYC_W2 = 4.05    # per SIMD with two or more waves sharing it (the MD5 mix, tools/mb/valu_mix.hip)


def issue_compute(path, key, launch_s, dispatches=1):
    """roofline.compute for the lines bound by instruction issue rather than by HBM: one wave per
    SIMD (RC4 and frame/open, variable-length digests) or one producer / consumer wave pair per
    SIMD (MetaData unpack, segment digests; both waves' instructions count); VERDICT r03 item 4.  From the kept --pmc pass of the same kernel
    (per dispatch; `dispatches` per step):
      issued_per_simd  (SQ_INSTS_VALU + SQ_INSTS_LDS + SQ_INSTS_SALU) / 1024 SIMDs
      frac_issue_ceiling  issued_per_simd x cycles per instruction / (launch time x CLOCK_GHZ): the
                       share of the launch the SIMD needs just to issue those instructions at the
                       measured rate -- ISSUE_CYC_LONE for one wave per SIMD, ISSUE_CYC_W2 for two or
                       more (1.0 = issue-bound with no slack);
      issue_busy_frac  SQ_ACTIVE_INST_ANY x 4 / 1024 / (GRBM_GUI_ACTIVE / 8): the share of dispatch
                       cycles each SIMD had a wave issuing (clock-free);
      wait_frac / wait_inst_frac  SQ_WAIT_ANY / SQ_WAVE_CYCLES (waiting on memory or LDS data) and
                       SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (waiting for an issue slot)."""
    _, det, why = load_pmc(path, key)
    if why:
        return {"refused": why}
    if "sq_insts_valu" not in det:
        return None
    per_launch = launch_s / dispatches
    insts = det["sq_insts_valu"] + det.get("sq_insts_lds", 0) + det.get("sq_insts_salu", 0)
    per_simd = insts / SIMDS
    wps = det.get("sq_waves", SIMDS) / SIMDS            # waves per SIMD (every wave resident at once here)
    cyc = ISSUE_CYC_LONE if wps < 1.5 else ISSUE_CYC_W2
    out = {"bound": "simd issue", "issued_per_simd": round(per_simd, 1),
           "valu_per_simd": round(det["sq_insts_valu"] / SIMDS, 1), "waves_per_simd": round(wps, 2),
           "cycles_per_inst": cyc, "clock_ghz": CLOCK_GHZ,
           "frac_issue_ceiling": round(per_simd * cyc / (per_launch * CLOCK_GHZ * 1e9), 4),
           "source": det.get("source"), "kernels": det.get("kernels")}
    if "sq_active_inst_any" in det and det.get("grbm_gui_active"):
        out["issue_busy_frac"] = round(det["sq_active_inst_any"] * 4 / SIMDS / (det["grbm_gui_active"] / 8), 4)
    if det.get("sq_wave_cycles"):
        out["wait_frac"] = round(det.get("sq_wait_any", 0) / det["sq_wave_cycles"], 4)
        out["wait_inst_frac"] = round(det.get("sq_wait_inst_any", 0) / det["sq_wave_cycles"], 4)
    return out


def main():
    args = parse()
    if args.config == 1:          # plumbing, no GPU (BASELINE cfg1)
        print(json.dumps(bench_cfg1(args)), flush=True)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "RANK" not in os.environ:
        relaunch_distributed(args)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import numpy as np
    import torch

    import brb_framework_amd as brb
    from brb_framework_amd import workload

    # one process per GPU; RCCL ("nccl") for the barrier and the max-over-ranks.  Only when ranks
    # outnumber the visible GPUs (a rehearsal of --gpus 2 on a one-GPU box) do they share a card and
    # use gloo (RCCL refuses two ranks on one device).
    ndev = torch.cuda.device_count()
    torch.cuda.set_device(local_rank % ndev)
    dev = torch.device("cuda", local_rank % ndev)
    dist = None
    backend = "nccl" if world <= ndev else "gloo"
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    if not brb.gpu_available():
        raise SystemExit("libbrb_crypto_gpu: " + brb.lib().BRB_CryptoGPU_LastError().decode())
    for opt in args.test_option:
        name, value = opt.split("=")
        brb.test_option(name, int(value))

    def opt_value(name):
        old = brb.test_option(name, 0)     # every option's range holds 0
        brb.test_option(name, old)
        return old
    global MARK, OPT
    OPT = opt_value
    MARK = args.mark_timed_region

    def barrier():
        if dist is not None:
            dist.barrier()

    def max_over_ranks(x: float) -> float:
        if dist is None:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def log(msg):
        if rank == 0:
            print(msg, file=sys.stderr, flush=True)

    cfg_id = args.config
    cfg = workload.CONFIGS[cfg_id]
    stream = torch.cuda.current_stream(dev)

    if args.op == "batcher":
        result = bench_batcher(args, rank, world, log)
    elif args.op in ("rc4", "rc4md5"):
        result = bench_rc4(args, rank, world, dev, stream, barrier, max_over_ranks, log)
    elif args.op in ("md5var", "sha1var"):
        result = bench_var(args, rank, world, dev, stream, barrier, max_over_ranks, log)
    elif args.op in ("metadata", "md5seg", "base64"):
        result = bench_f4(args, rank, world, dev, stream, barrier, max_over_ranks, log)
    elif cfg["op"] == "blowfish":
        result = bench_blowfish(args, cfg, rank, world, dev, stream, barrier, max_over_ranks, log)
    else:
        result = bench_digest(args, cfg_id, cfg, rank, world, dev, stream, barrier, max_over_ranks, log)
    if rank == 0:
        if NOTES:
            result["notes"] = NOTES
        if SETTLE and "settle" not in result:
            result["settle"] = SETTLE
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


# ------------------------------------------------------------------------------------------------
def warm_up(args, launch, streams, torch, max_over_ranks, warm_s=1.0, timed_s=0.3):
    """W untimed steps, then the choice of K.  Explicit --warmup / --steps are used as given.  By
    default the GPU is kept busy for >= warm_s before timing: a fresh MI355X starts at a low clock
    and ramps over hundreds of ms (cfg2 MD5: 30.4 us per launch after 20 warm-up steps, 25.4 us at
    steady state), and K fills >= timed_s of GPU time.  Step k goes to streams[k % len(streams)].
    Returns (W, K); K is the same on every rank (max over ranks)."""
    global SETTLE
    n = 0
    step_s = None
    if args.warmup is not None:
        # settle: the same launches for >= warm_s before the W steps, so a short W (the driver passes
        # --warmup 5, 0.1 ms of GPU work) does not leave the timed region at a clock still moving:
        # after the cfg5 leg or on a fresh box the first K = 20 launches ran 22.1 us against 20.5 us
        # settled (tools/gpu_short_bench.sh, profiles/r05/short/).  Untimed, like the W steps; the
        # timed region is still exactly K steps.  Recorded on the line as "settle".
        # With several ranks the settle ends together on all of them, so that no GPU idles at the
        # region's barrier waiting for a slower rank (an idle spell is what the settle is against):
        # the timed part (chunks of <= 20 ms, so ranks leave it within one chunk) is followed by a
        # collective that agrees the launch time, then ~50 ms of the same number of launches on
        # every rank.
        settle_s = getattr(args, "settle_s", warm_s)
        if settle_s > 0:
            max_over_ranks(0.0)                     # a collective: the ranks start the settle together
        t0, chunk, m, dt = time.perf_counter(), 4, 0, None
        while time.perf_counter() - t0 < settle_s:
            tc = time.perf_counter()
            for _ in range(chunk):
                launch(m, streams[m % len(streams)], m % len(streams))
                m += 1
            torch.cuda.synchronize()
            dt = (time.perf_counter() - tc) / chunk
            chunk = min(chunk * 2, max(4, int(0.02 / max(dt, 1e-7))))
        if dt is not None:
            tail = max(4, math.ceil(0.05 / max(max_over_ranks(dt), 1e-7)))
            for _ in range(tail):
                launch(m, streams[m % len(streams)], m % len(streams))
                m += 1
            torch.cuda.synchronize()
        SETTLE = None if m == 0 else {"launches": m, "seconds": round(time.perf_counter() - t0, 3),
                  "why": "untimed launches of the same step before the W warm-up steps, so the timed region "
                         "starts at the clock the chip holds under this load (a short W does not reach it)"}
        for k in range(args.warmup):
            launch(k, streams[k % len(streams)], k % len(streams))
        torch.cuda.synchronize()
        n = args.warmup
    else:
        t0, chunk = time.perf_counter(), 4
        while True:
            tc = time.perf_counter()
            for _ in range(chunk):
                launch(n, streams[n % len(streams)], n % len(streams))
                n += 1
            torch.cuda.synchronize()
            step_s = (time.perf_counter() - tc) / chunk
            if time.perf_counter() - t0 >= warm_s:
                break
            chunk = min(chunk * 2, max(4, int(0.1 / max(step_s, 1e-7))))
    if args.steps is not None:
        k = args.steps
    else:
        if step_s is None:
            tc = time.perf_counter()
            for _ in range(8):
                launch(n, streams[n % len(streams)], n % len(streams))
                n += 1
            torch.cuda.synchronize()
            step_s = (time.perf_counter() - tc) / 8
        k = max(200, math.ceil(timed_s / step_s))
    return n, int(max_over_ranks(float(k)))


SETTLE = None    # warm_up(): the untimed settle before an explicit W (attached to the line)
MARK = False     # --mark-timed-region
LAST_ALL_K_S = None   # per-launch seconds of the last timed region over ALL K launches (events)


def timed_steps(launch, n_steps, streams, barrier, max_over_ranks, torch):
    """K steps between barrier + synchronize on both sides; step k is enqueued on
    streams[k % len(streams)] straight through the C ABI (pre-resolved ctypes arguments, so the
    host enqueues faster than the GPU drains).  Returns (wall seconds max over ranks, seconds per
    launch from HIP events on the launch stream).

    The per-launch time is what roofline.achieved divides by.  On one stream with K >= 3 the event
    pair brackets steps 3..K: e0 is enqueued right after step 2 (it fires when step 2 ends), e1
    when step K ends -- K-2 back-to-back launches.  Left out: the host-to-GPU latency of the first
    launch, and the first two launches after the idle synchronize, which run 15-25 % slower (a
    20-step region under rocprofv3: 25.2 and 27.2 us, then 21.5-22.8 us).  Recording e0 after step
    2 rather than step 1 also keeps the host's event call off the critical path: enqueued between
    steps 1 and 2 it left a 5.6 us gap between the two kernels.  The wall time (and so `value`)
    covers all K steps.  Nothing is enqueued between kernels.  LAST_ALL_K_S keeps the same events'
    time over all K launches (an event recorded before step 0), the round-2 method, so the two can be
    compared.
    """
    global LAST_ALL_K_S
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ea = torch.cuda.Event(enable_timing=True)
    if MARK:             # sentinel before the region, drained before t0
        with torch.cuda.stream(streams[0]):
            torch.cuda._sleep(1)
    steady = len(streams) == 1 and n_steps >= 3
    for e in (ea, e0, e1):   # torch creates a HIP event at its first record: not inside the region
        e.record(streams[0])
    gc_was = gc.isenabled()
    gc.disable()         # no collector pause inside a region of a few hundred microseconds
    try:                 # a raise inside the region must not leave the collector off
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if steady:
            ea.record(streams[0])
        else:
            e0.record(streams[0])
        for k in range(n_steps):
            j = k % len(streams)
            launch(k, streams[j], j)
            if steady and k == 1:
                e0.record(streams[0])
        e1.record(streams[0])
        torch.cuda.synchronize()
        barrier()
        t1 = time.perf_counter()
    finally:
        if gc_was:
            gc.enable()
    if MARK:             # sentinel after the region, enqueued after the timing ended
        with torch.cuda.stream(streams[0]):
            torch.cuda._sleep(1)
        torch.cuda.synchronize()
    wall = max_over_ranks(t1 - t0)
    LAST_ALL_K_S = ((ea if steady else e0).elapsed_time(e1) / 1e3 / n_steps) if len(streams) == 1 else None
    return wall, e0.elapsed_time(e1) / 1e3 / (n_steps - 2 if steady else n_steps)


def bench_digest(args, cfg_id, cfg, rank, world, dev, stream, barrier, max_over_ranks, log):
    import numpy as np
    import torch

    import brb_framework_amd as brb
    from brb_framework_amd import workload

    L = args.rec_len or cfg["rec_len"]
    if cfg_id == 5:
        n_rank = workload.CONFIGS[5]["records"] // 8          # one GPU's shard of cfg5
    else:
        n_rank = cfg["records"]
    if args.records_per_gpu:
        n_rank = args.records_per_gpu
    n_global = n_rank * world
    r0 = rank * n_rank                                         # this rank's contiguous shard
    seed = workload.SEEDS[cfg_id]
    fn = brb.md5_batch_fixed if args.op == "md5" else brb.sha1_batch_fixed
    width = 16 if args.op == "md5" else 20

    t = time.perf_counter()
    host = workload.gen_records(seed, r0, n_rank, L)
    log(f"[bench] generated {host.nbytes / 1e6:.1f} MB on host in {time.perf_counter() - t:.1f}s")
    cfg5 = None
    if cfg_id == 2 and args.op == "md5" and not args.no_cfg5 and not args.records_per_gpu and not args.rec_len:
        # the cfg5 sub-measurement (>= 1.3 s of GPU work) runs BEFORE the headline's W warm-up steps:
        # a fresh MI355X starts at a low clock and takes hundreds of ms to reach its loaded state, which
        # a short W (the driver passes --warmup 5 = 0.1 ms) does not cover (r02: 22.46 us per launch
        # after 5 warm-up steps, 20.99 us in steady state).  It also runs before the headline's
        # batches are copied to the device (milliseconds, so the clock stays up), so its 1.57 GB
        # sweep does not come between those buffers' first writes and their first timed reads.  The
        # order changes no work and no timing rule: each region is still W untimed + K timed steps
        # between barrier + synchronize.
        cfg5, cfg5_verify = bench_cfg5(args, rank, world, dev, stream, barrier, max_over_ranks, log)
        # (its digest check runs after the headline's timed region: no idle gap between the legs)
    batch_bytes = host.nbytes
    n_rot = max(2, math.ceil(640e6 / batch_bytes)) if batch_bytes < 2.5 * L3_BYTES else 1
    bufs = [torch.from_numpy(host).to(dev)]
    for _ in range(n_rot - 1):
        bufs.append(bufs[0].clone())
    n_streams = max(1, args.streams)
    outs = [torch.empty((n_rank, width), dtype=torch.uint8, device=dev) for _ in range(max(2, n_streams) + 1)]
    torch.cuda.synchronize()
    # dedicated non-default streams for the multi-stream runs (the legacy default stream would
    # serialise with them)
    side = [torch.cuda.Stream(dev) for _ in range(max(2, n_streams))]
    all_streams = [stream] + side

    def launch(k, s, j=0):
        fn(bufs[k % n_rot], L, n_rank, out=outs[j], stream=s, async_=True)

    # raw C-ABI launcher: all pointers resolved once (what a C caller pays per call)
    cfn = brb.lib().BRB_MD5BatchFixed if args.op == "md5" else brb.lib().BrbSha1_BatchFixed
    buf_ptrs = [b.data_ptr() for b in bufs]
    out_ptrs = [o.data_ptr() for o in outs]
    flags = brb.BATCH_DEVICE | brb.BATCH_ASYNC

    def launch_raw(k, s, j=0):
        rc = cfn(buf_ptrs[k % n_rot], L, n_rank, out_ptrs[j], flags, s.cuda_stream)
        if rc != 1:
            raise RuntimeError(brb.lib().BRB_CryptoGPU_LastError().decode())

    for j, s_ in enumerate(all_streams):                        # one eager call per stream
        launch(j, s_, j)
    main_streams = [stream] if n_streams == 1 else side[:n_streams]
    # warm up on the streams the timed region uses (so rocprof's per-kernel average over the whole
    # run describes the same back-to-back launches as the timed region)
    n_warm, n_steps = warm_up(args, launch_raw, main_streams, torch, max_over_ranks)
    wall, ev_s = timed_steps(lambda k, s, j: launch_raw(k + n_warm, s, j), n_steps, main_streams,
                             barrier, max_over_ranks, torch)
    all_k_s = LAST_ALL_K_S
    if cfg5 is not None:
        cfg5_verify()
    wall2 = None
    if args.two_stream:
        # the same K steps alternating over two HIP streams (two batches in flight)
        wall2, _ = timed_steps(launch_raw, n_steps, side[:2], barrier, max_over_ranks, torch)
    out = outs[0]

    # spot-check the last step's digests against hashlib (stdlib, independent of this repo)
    got = out.cpu().numpy()
    h = hashlib.md5 if args.op == "md5" else hashlib.sha1
    for i in list(np.random.default_rng(rank).integers(0, n_rank, 32)) + [0, n_rank - 1]:
        assert got[i].tobytes() == h(host[i * L:(i + 1) * L].tobytes()).digest(), f"digest mismatch at {i}"

    total_bytes = n_global * L * n_steps
    gib_s = total_bytes / wall / 2**30
    mrec_s = n_global * n_steps / wall / 1e6
    # per-launch duration from the events around the timed region (single stream: launches run back
    # to back, so this is the kernel time plus the ~2 us dependent-kernel boundary)
    avg_kern_s = ev_s
    achieved = n_rank * L / avg_kern_s / 1e9
    pmc_key = f"cfg{cfg_id}_{args.op}"
    result = {
        "metric": METRIC,
        "value": round(gib_s, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": n_steps,
        "warmup": n_warm,
        "ms_per_step": round(wall / n_steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (SURVEY §8(d) splitmix64 generator, HBM-resident, L3-defeating rotation of "
                f"{n_rot} copies)",
        "config": {"workload": ((cfg["name"] if args.op == "md5" else cfg["name"].replace(" MD5", " SHA-1") + " (SHA-1 on the "
                                 f"cfg{cfg_id} shape; BASELINE's digest is MD5)")
                                if not args.rec_len else f"{n_rank} x {L} B records (cfg{cfg_id} shape, --rec-len)")
                   + (f" (shard of {n_rank} records/GPU)" if cfg_id == 5 else "")
                   + (f"; the same batch on each of {world} GPUs" if world > 1 and cfg_id != 5 else ""),
                   "op": f"{'BRB_MD5BatchFixed' if args.op == 'md5' else 'BrbSha1_BatchFixed'} (device mode)",
                   "records_per_gpu": n_rank, "record_bytes": L, "global_records": n_global,
                   "parallelism": f"record-shard x{world}, no collective"},
        "mrecords_per_s": round(mrec_s, 3),
        "streams": n_streams,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), **traffic_fields(args.pmc_summary, pmc_key),
                     "launch_us_avg": round(avg_kern_s * 1e6, 2), "bytes_per_launch": n_rank * L,
                     "launch_us_avg_all_k": round(all_k_s * 1e6, 2) if all_k_s else None,
                     "frac_all_k": round(n_rank * L / all_k_s / 1e9 / HBM_PEAK_GBS, 4) if all_k_s else None,
                     "timing": TIMING,
                     "compute": compute_fraction(args.pmc_summary, pmc_key, avg_kern_s,
                                                 LONE_WAVE_CYC.get(args.op) if n_rank <= 65536 else None)},
    }
    if wall2 is not None:
        result["two_stream_throughput"] = {
            "value": round(n_global * L * n_steps / wall2 / 2**30, 2), "unit": "GiB/s",
            "mrecords_per_s": round(n_global * n_steps / wall2 / 1e6, 3),
            "note": "same K steps alternating over 2 HIP streams (2 batches in flight)"}
    if world == 1 and not args.no_pcie:
        result["pcie_inclusive"] = bench_pcie_digest(fn, host, L, n_rank, width, log)
    del bufs, outs
    torch.cuda.empty_cache()
    if cfg5 is not None:
        result["cfg5"] = cfg5
        result["order"] = ("cfg5 sub-measurement first (GPU at its loaded clock), then the headline's batches copied to "
                           "the device, its W warm-up + K timed steps, then the host-inclusive and CPU legs")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_digest(args, host, L, n_rank, log)
    log(f"[bench] launch avg {avg_kern_s * 1e6:.1f} us -> {achieved:.0f} GB/s ({achieved / HBM_PEAK_GBS:.1%} of HBM peak)")
    return result


def host_rate(call, nbytes, reps=5):
    """Mean wall time of `call` (after one untimed call that sizes the library's scratch)."""
    call()
    t = time.perf_counter()
    for _ in range(reps):
        call()
    dt = (time.perf_counter() - t) / reps
    return {"gib_s": round(nbytes / dt / 2**30, 2), "gb_s": round(nbytes / dt / 1e9, 2), "ms": round(dt * 1e3, 3)}


def registered_copy(arr):
    """A copy of `arr` in page-aligned host memory page-locked with BRB_CryptoGPU_HostRegister (what a
    C caller does with its own buffers); returns (region, numpy view).  Delete the view, then
    region.close()."""
    import numpy as np

    import brb_framework_amd as brb
    reg = brb.crypto.HostRegion(arr.nbytes)
    view = np.frombuffer(reg._mm, np.uint8, count=arr.nbytes).view(arr.dtype).reshape(arr.shape)
    view[...] = arr
    return reg, view


def bench_pcie_digest(fn, host, L, n, width, log):
    """Host-inclusive rate through the C ABI's host mode (input in host memory, digests back in host
    memory, the call returns when they are there): pageable input (a plain numpy array, what a
    receive loop's calloc'd buffers are), page-locked input (the same bytes in a region the library
    page-locked, BRB_CryptoGPU_HostRegister) and torch.pin_memory() input for comparison."""
    import numpy as np
    import torch
    out = np.empty((n, width), np.uint8)
    pageable = host_rate(lambda: fn(host, L, n, out=out), host.nbytes)
    reg, hp = registered_copy(host)
    pinned = host_rate(lambda: fn(hp, L, n, out=out), host.nbytes)
    del hp
    reg.close()
    tp = torch.from_numpy(host).pin_memory().numpy()
    pinned_torch = host_rate(lambda: fn(tp, L, n, out=out), host.nbytes)
    log(f"[bench] host-inclusive: pageable {pageable['gb_s']} GB/s, page-locked {pinned['gb_s']} GB/s, "
        f"torch-pinned {pinned_torch['gb_s']} GB/s")
    return {"gib_s": pageable["gib_s"], "ms_per_batch": pageable["ms"], "pageable": pageable, "pinned": pinned,
            "pinned_torch": pinned_torch,
            "note": "host-mode call: 32 MiB chunks of whole records copied H2D straight from the caller's memory, overlapped "
                    "with the kernels, digests D2H per chunk; gib_s = pageable input"}


def bench_cfg5(args, rank, world, dev, stream, barrier, max_over_ranks, log):
    """BASELINE cfg5: 8 388 608 x 1500 B records sharded by contiguous ranges over 8 GPUs, 1 048 576
    per GPU (no collective).  Every rank digests records [rank * 2^20, (rank + 1) *
    2^20) of the cfg5 generator; at world 8 the job is exactly cfg5, at other N the same per-GPU
    shard (weak scaling).  >= 1 s of warm-up, then K steps (>= 0.3 s) between barrier + synchronize,
    max over ranks; 1.57 GB per
    shard defeats the 256 MiB Infinity Cache by itself.  Both ends of each shard are checked
    against the hashlib golden digests (tests/golden/digests.json configs["5"])."""
    import numpy as np
    import torch

    import brb_framework_amd as brb
    from brb_framework_amd import workload

    L = workload.CONFIGS[5]["rec_len"]
    n = workload.CONFIGS[5]["records"] // 8
    r0 = rank * n
    t = time.perf_counter()
    host = workload.gen_records(workload.SEEDS[5], r0, n, L)
    log(f"[bench] cfg5: generated {host.nbytes / 1e9:.2f} GB per GPU in {time.perf_counter() - t:.1f}s")
    buf = torch.from_numpy(host).to(dev)
    out = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    cfn = brb.lib().BRB_MD5BatchFixed
    flags = brb.BATCH_DEVICE | brb.BATCH_ASYNC

    def launch(k, s, j=0):
        if cfn(buf.data_ptr(), L, n, out.data_ptr(), flags, s.cuda_stream) != 1:
            raise RuntimeError(brb.lib().BRB_CryptoGPU_LastError().decode())

    # the clock ramps down while the host-inclusive leg runs: warm up >= 1 s like the main steps
    _, steps = warm_up(argparse.Namespace(warmup=None, steps=None), launch, [stream], torch, max_over_ranks)
    wall, ev_s = timed_steps(launch, steps, [stream], barrier, max_over_ranks, torch)
    launch_s = ev_s
    buf = None                                   # the digests stay for verify(); 1.57 GB go back
    total = n * world
    log(f"[bench] cfg5: {launch_s * 1e6:.1f} us per 1 Mi-record launch")
    res = {}

    def verify():
        """The shard's digests against the golden file and hashlib (run after the headline's timed
        region, so the host-side check leaves no idle gap between the two GPU legs)."""
        nonlocal out
        got = out.cpu().numpy()
        with open(os.path.join(ROOT, "tests", "golden", "digests.json")) as f:
            gold = json.load(f)["configs"]["5"]["digests"]
        checked = 0
        for e in gold:
            if r0 <= e["r"] < r0 + n:
                assert got[e["r"] - r0].tobytes().hex() == e["md5"], f"cfg5 digest mismatch at record {e['r']}"
                checked += 1
        for i in np.random.default_rng(rank + 5).integers(0, n, 16):
            assert got[i].tobytes() == hashlib.md5(host[i * L:(i + 1) * L].tobytes()).digest()
        res["golden_checked_on_rank0"] = checked if rank == 0 else None
        out = None
        torch.cuda.empty_cache()

    res.update({"workload": "cfg5: 8388608 x 1500 B MD5, record-sharded over 8 GPUs" if world == 8 else
                        f"cfg5 shard shape: {n} x 1500 B MD5 per GPU x {world} GPU(s) (exactly cfg5 at --gpus 8)",
            "records_total": total, "records_per_gpu": n, "steps": steps,
            "value": round(total * L * steps / wall / 2**30, 2), "unit": "GiB/s",
            "mrecords_per_s": round(total * steps / wall / 1e6, 3), "ms_per_step": round(wall / steps * 1e3, 4),
            "launch_us_avg": round(launch_s * 1e6, 2),
            "roofline_frac": round(n * L / launch_s / 1e9 / HBM_PEAK_GBS, 4),
            "note": "per-GPU shard of 1 048 576 records; wall time max over ranks"})
    return res, verify


def cpu_baseline_digest(args, host, L, n, log):
    import oracle     # test infrastructure: the CPU restatement is the baseline, never the product
    threads = cpu_threads()
    fn = oracle.md5_batch_fixed if args.op == "md5" else oracle.sha1_batch_fixed
    res = {}
    for th in (threads, 1):
        n_s = n if th > 1 else max(1, n // 16)
        fn(host, L, min(n_s, 1024), threads=th)
        reps, t0 = 0, time.perf_counter()
        while True:
            fn(host, L, n_s, threads=th)
            reps += 1
            if time.perf_counter() - t0 >= args.cpu_seconds / 2:
                break
        dt = time.perf_counter() - t0
        res[th] = (n_s * L * reps / dt / 2**30, reps, n_s)
    gib, reps, n_s = res[threads]
    log(f"[bench] cpu baseline {gib:.2f} GiB/s on {threads} threads, {res[1][0]:.3f} GiB/s on 1")
    return {"value": round(gib, 3), "unit": "GiB/s", "kind": "port",
            **core_counts(threads, res[1][0]),
            "sample": f"oracle/brb_oracle.c {args.op} over the same {n_s} x {L} B records, {reps} passes, "
                      f"{threads} pthreads (-O2 as libbrb_core/Makefile.linux:3)",
            "single_core_gib_s": round(res[1][0], 4)}


# ------------------------------------------------------------------------------------------------
def bench_blowfish(args, cfg, rank, world, dev, stream, barrier, max_over_ranks, log):
    """cfg4: 65 536 x 16 KiB records, Blowfish encrypt then decrypt (one ctx), per GPU."""
    import numpy as np
    import torch

    import brb_framework_amd as brb
    from brb_framework_amd import workload
    import oracle

    n_rec = args.records_per_gpu or cfg["records"]
    n_words = n_rec * cfg["rec_len"] // 8
    n_blocks = n_words // 2
    ctx = brb.blowfish_init(workload.CFG4_KEY)
    cdev = torch.frombuffer(bytearray(brb.blowfish_ctx_bytes(ctx)), dtype=torch.uint8).to(dev)
    t = time.perf_counter()
    w = workload.gen_words(workload.SEEDS[4], n_words, r0=rank * n_words)
    log(f"[bench] generated {w.nbytes / 1e6:.0f} MB of plaintext in {time.perf_counter() - t:.1f}s")
    d = torch.from_numpy(w.view(np.int64)).to(dev)
    d0 = d.clone()
    ev_enc = []

    def launch(k, s, j=0):
        brb.blowfish_encrypt_batch(cdev, d, n_blocks, stream=s, async_=True)
        brb.blowfish_decrypt_batch(cdev, d, n_blocks, stream=s, async_=True)

    n_warm, n_steps = warm_up(args, launch, [stream], torch, max_over_ranks)
    wall, ev_s = timed_steps(launch, n_steps, [stream], barrier, max_over_ranks, torch)
    assert torch.equal(d, d0), "Blowfish round trip did not restore the plaintext"
    # one encrypt-only check against the oracle on a sample record
    brb.blowfish_encrypt_batch(cdev, d, n_blocks)
    wpr = cfg["rec_len"] // 8
    got = d[:wpr].cpu().numpy().view(np.uint64)
    assert np.array_equal(got, oracle.bf_ecb(oracle.bf_init(workload.CFG4_KEY), w[:wpr].copy()))
    step_s = ev_s
    plain = n_words * 8
    result = {
        "metric": "GiB/s of plaintext per Blowfish encrypt+decrypt round trip (cfg4)",
        "value": round(plain * world * n_steps / wall / 2**30, 2),
        "unit": "GiB/s",
        "n_gpus": world, "steps": n_steps, "warmup": n_warm,
        "ms_per_step": round(wall / n_steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic (splitmix64 words, HBM-resident)",
        "config": {"workload": cfg["name"], "records_per_gpu": n_rec, "record_bytes": cfg["rec_len"],
                   "parallelism": f"record-shard x{world}, no collective"},
        "roofline": {"bound": "hbm", "achieved": round(4 * plain / step_s / 1e9, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(4 * plain / step_s / 1e9 / HBM_PEAK_GBS, 4),
                     **traffic_fields(args.pmc_summary, "cfg4_blowfish", per_step=2),
                     "step_us_avg": round(step_s * 1e6, 2), "bytes_per_step": 4 * plain,
                     "note": "algorithmic bytes = read + write of the plaintext in each direction",
                     "compute": blowfish_compute(args.pmc_summary)},
    }
    if world == 1 and not args.no_pcie:
        result["pcie_inclusive"] = bench_pcie_blowfish(ctx, w, log)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        oc = oracle.bf_init(workload.CFG4_KEY)
        th = cpu_threads()
        sample = w[: min(n_words, 2 * 1024 * 1024)].copy()
        reps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < args.cpu_seconds:
            oracle.bf_ecb(oc, sample, threads=th)
            oracle.bf_ecb(oc, sample, decrypt=True, threads=th)
            reps += 1
        dt = time.perf_counter() - t0
        one = sample[: len(sample) // 16].copy()
        t1 = time.perf_counter()
        oracle.bf_ecb(oc, one)
        oracle.bf_ecb(oc, one, decrypt=True)
        single = one.nbytes / (time.perf_counter() - t1) / 2**30
        result["cpu_baseline"] = {"value": round(sample.nbytes * reps / dt / 2**30, 3), "unit": "GiB/s",
                                  "kind": "port", **core_counts(th, single),
                                  "single_core_gib_s": round(single, 4),
                                  "sample": f"oracle bf_ecb enc+dec over {sample.nbytes >> 20} MiB, {reps} passes, "
                                            f"{th} pthreads"}
    return result


def blowfish_compute(path):
    """roofline.compute for bf_rep_kernel: SIMD instruction issue bounds it (every SIMD issues on
    ~100 % of the cycles at ~4 cycles per instruction: 11 VALU + 4 LDS gathers per F), the LDS gathers
    come second.  SQ_LDS_IDX_ACTIVE counts LDS-busy cycles summed over the 256 CUs (checked: 2.0 per
    ds_read_b32 in the MD5 kernel, 3.0 per ds_read_b64 here = 2 + its one 2-way bank conflict), and
    GRBM_GUI_ACTIVE / 8 is the dispatch's busy cycles per XCD (reliable on dispatches over 0.3 ms,
    MI355X_MICROARCH.md "DVFS give-back"), so lds_busy_frac = (IDX_ACTIVE / 256) / (GUI_ACTIVE / 8)
    with no clock assumption; valu_frac_peak = SQ_INSTS_VALU / 1024 SIMDs x 2 cycles over the same
    cycles."""
    _, det, why = load_pmc(path, "cfg4_blowfish")
    if why:
        return {"refused": why}
    if "sq_lds_idx_active" not in det or "grbm_gui_active" not in det:
        return None
    cyc = det["grbm_gui_active"] / 8
    out = {"bound": "simd-issue, then lds-gather", "dispatch_cycles": round(cyc),
           "lds_busy_frac": round(det["sq_lds_idx_active"] / 256 / cyc, 4),
           "lds_bank_conflict_frac": round(det.get("sq_lds_bank_conflict", 0) / 256 / cyc, 4),
           "valu_frac_peak": round(det["sq_insts_valu"] / SIMDS * VALU_PEAK_CYC / cyc, 4),
           "source": det.get("source"), "kernels": det.get("kernels")}
    if "sq_active_inst_any" in det:
        # SQ_ACTIVE_INST_ANY: quad-cycles in which a wave issued, summed over waves; x 4 / 1024 SIMDs
        # = the cycles each SIMD spent issuing (4 waves per SIMD here, at most one issuing at a time)
        out["issue_busy_frac"] = round(det["sq_active_inst_any"] * 4 / SIMDS / cyc, 4)
        insts = det["sq_insts_valu"] + det.get("sq_insts_lds", 0) + det.get("sq_insts_salu", 0)
        out["cycles_per_issued_inst"] = round(det["sq_active_inst_any"] * 4 / insts, 2)
    return out


def bench_pcie_blowfish(ctx, w, log):
    """cfg4 host-inclusive: the 1 GiB of words in host memory, encrypted then decrypted in place by
    two host-mode calls (every byte crosses PCIe four times per round trip); pageable and
    page-locked.  Rate = plaintext bytes per round trip."""
    import torch

    import brb_framework_amd as brb
    buf = w.copy()

    def trip(b):
        brb.blowfish_encrypt_batch(ctx, b)
        brb.blowfish_decrypt_batch(ctx, b)

    pageable = host_rate(lambda: trip(buf), w.nbytes, reps=3)
    reg, pb = registered_copy(buf)
    pinned = host_rate(lambda: trip(pb), w.nbytes, reps=3)
    assert (pb == w).all() and (buf == w).all(), "host-mode round trip did not restore the plaintext"
    del pb
    reg.close()
    log(f"[bench] cfg4 host-inclusive: pageable {pageable['gib_s']} GiB/s, pinned {pinned['gib_s']} GiB/s")
    return {"gib_s": pageable["gib_s"], "ms_per_round_trip": pageable["ms"], "pageable": pageable, "pinned": pinned,
            "note": "two host-mode calls (encrypt, decrypt) over the 1 GiB in place: 16 MiB chunks, H2D on the calling "
                    "thread and D2H on the device's worker thread overlap each other and the kernels"}


# ------------------------------------------------------------------------------------------------
def bench_cfg1(args):
    """BASELINE cfg1 (plumbing, no GPU): one 1 048 576-byte buffer through the product's compat
    BRB_MD5Init / BRB_MD5UpdateBig / BRB_MD5Final (md5.c:38-168) on one CPU thread, the digest
    checked against the hashlib golden digest; the oracle's MD5 of the same buffer is timed beside
    it as the CPU baseline."""
    import ctypes

    import brb_framework_amd as brb
    from brb_framework_amd import workload
    import oracle

    L = brb.lib()
    cfg = workload.CONFIGS[1]
    buf = workload.gen_records(workload.SEEDS[1], 0, 1, cfg["rec_len"]).tobytes()
    with open(os.path.join(ROOT, "tests", "golden", "digests.json")) as f:
        want = json.load(f)["configs"]["1"]["digests"][0]["md5"]
    ctx = brb.BRB_MD5_CTX()

    def compat():
        L.BRB_MD5Init(ctypes.byref(ctx))
        L.BRB_MD5UpdateBig(ctypes.byref(ctx), buf, len(buf))
        L.BRB_MD5Final(ctypes.byref(ctx))

    def timed(fn, seconds, k=None, w=1):
        """W untimed calls, then exactly K timed ones (--steps / --warmup), or as many as fill
        `seconds`."""
        for _ in range(max(1, w)):
            fn()
        n, t0 = 0, time.perf_counter()
        while (n < k) if k else (time.perf_counter() - t0 < seconds):
            fn()
            n += 1
        return n, time.perf_counter() - t0

    warm = args.warmup if args.warmup is not None else 1
    steps, dt = timed(compat, max(1.0, args.cpu_seconds / 2), args.steps, warm)
    assert bytes(ctx.digest).hex() == want, "compat MD5 of the cfg1 buffer differs from the golden digest"
    o_steps, o_dt = timed(lambda: oracle.md5(buf), max(1.0, args.cpu_seconds / 2))
    assert oracle.md5(buf).hex() == want
    rate = len(buf) * steps / dt / 2**30
    o_rate = len(buf) * o_steps / o_dt / 2**30
    return {"metric": "GiB/s of MD5 over one 1 MiB buffer through the compat BRB_MD5Init/UpdateBig/Final (cfg1, CPU)",
            "value": round(rate, 3), "unit": "GiB/s", "n_gpus": 0, "steps": steps, "warmup": max(1, warm),
            "ms_per_step": round(dt / steps * 1e3, 4), "higher_is_better": True, "scaling": "none",
            "vs_baseline": None, "dtype": "u32", "data": "synthetic (SURVEY §8(d) generator, seed 0x5EED0001)",
            "config": {"workload": cfg["name"], "op": "BRB_MD5Init + BRB_MD5UpdateBig + BRB_MD5Final (compat, host C)",
                       "record_bytes": len(buf), "parallelism": "one CPU thread"},
            "digest": bytes(ctx.digest).hex(), "golden_match": True,
            "roofline": None,
            "cpu_baseline": {"value": round(o_rate, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
                             "sample": f"oracle/brb_oracle.c MD5 of the same 1 MiB buffer, {o_steps} passes"},
            "note": "cfg1 is the reference's single-buffer CPU path (SURVEY §8(d)): a serial chain of 16 385 "
                    "compressions, no GPU and no roofline"}


# ------------------------------------------------------------------------------------------------
def bench_rc4(args, rank, world, dev, stream, barrier, max_over_ranks, log):
    """SURVEY §8 f1 on the cfg2 shape: 65 536 connections x 1500-byte payloads per GPU.
    --op rc4:    one step = BRB_RC4_CryptBatch in place over every connection's buffer.
    --op rc4md5: one step = BRB_RC4MD5_FrameBatch (write side) of every payload into a 1530-byte
                 frame, then BRB_RC4MD5_OpenBatch (read side + validation) of those frames.
    The RC4 states advance from step to step exactly as a connection's stream does."""
    import numpy as np
    import torch

    import brb_framework_amd as brb
    from brb_framework_amd import workload
    import oracle

    L = 1500
    n = args.records_per_gpu or 65536
    H = brb.RC4MD5_HEADER
    host = workload.gen_records(workload.SEEDS[2], rank * n, n, L)
    n_rot = max(2, math.ceil(640e6 / host.nbytes))
    bufs = [torch.from_numpy(host).to(dev)]
    for _ in range(n_rot - 1):
        bufs.append(bufs[0].clone())
    rng = np.random.default_rng(rank)
    keys = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(n)]
    st0 = brb.rc4_states(keys)
    offs = torch.from_numpy(np.arange(n, dtype=np.uint64) * L).to(dev)
    lens = torch.full((n,), L, dtype=torch.int32, device=dev)
    FS = args.frame_stride or (L + H)
    assert FS >= L + H, "--frame-stride below the frame size"
    foffs = torch.from_numpy(np.arange(n, dtype=np.uint64) * FS).to(dev)
    flens = torch.full((n,), L + H, dtype=torch.int32, device=dev)
    salts = torch.from_numpy(rng.integers(0, 2**32, n, dtype=np.uint64)).to(dev)
    frames = torch.zeros(n * FS, dtype=torch.uint8, device=dev)
    valid = torch.zeros(n, dtype=torch.uint8, device=dev)
    wst, rst = torch.from_numpy(st0).to(dev), torch.from_numpy(st0).to(dev)
    Lb = brb.lib()
    flags = brb.BATCH_DEVICE | brb.BATCH_ASYNC
    P = {k: v.data_ptr() for k, v in dict(offs=offs, lens=lens, foffs=foffs, flens=flens, salts=salts,
                                           frames=frames, valid=valid, wst=wst, rst=rst).items()}
    bptr = [b.data_ptr() for b in bufs]

    def launch(k, s, j=0):
        h = s.cuda_stream
        if args.op == "rc4":
            rc = Lb.BRB_RC4_CryptBatch(P["wst"], bptr[k % n_rot], bptr[k % n_rot], P["offs"], P["lens"], n, flags, h)
        else:
            rc = Lb.BRB_RC4MD5_FrameBatch(P["wst"], bptr[k % n_rot], P["offs"], P["lens"], P["salts"], P["frames"],
                                          P["foffs"], n, flags, h)
            if rc == 1:
                rc = Lb.BRB_RC4MD5_OpenBatch(P["rst"], P["frames"], P["frames"], P["foffs"], P["flens"], n,
                                             P["valid"], flags, h)
        if rc != 1:
            raise RuntimeError(Lb.BRB_CryptoGPU_LastError().decode())

    n_warm, n_steps = warm_up(args, launch, [stream], torch, max_over_ranks)
    wall, ev_s = timed_steps(lambda k, s, j: launch(k + n_warm, s, j), n_steps, [stream], barrier,
                             max_over_ranks, torch)
    if args.op == "rc4md5":
        assert int(valid.sum()) == n, "a frame failed validation"
        assert torch.equal(wst, rst), "write and read states diverged"
        fr = frames[: 2 * (L + H)].cpu().numpy()
        assert fr[H:H + L].tobytes() == host[:L].tobytes()      # decrypted in place by the open step
    step_s = ev_s
    payload = n * L
    moved = 2 * payload if args.op == "rc4" else payload + 3 * n * (L + H)
    name = "BRB_RC4_CryptBatch" if args.op == "rc4" else "BRB_RC4MD5_FrameBatch + BRB_RC4MD5_OpenBatch"
    result = {
        "metric": f"GiB/s of payload per {'RC4 pass' if args.op == 'rc4' else 'RC4+MD5 frame + open round trip'} "
                  "(SURVEY §8 f1)",
        "value": round(payload * world * n_steps / wall / 2**30, 2),
        "unit": "GiB/s", "n_gpus": world, "steps": n_steps, "warmup": n_warm,
        "ms_per_step": round(wall / n_steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8",
        "data": f"synthetic (splitmix64 payloads, HBM-resident, {n_rot} rotating copies; random 16-byte keys)",
        "config": {"workload": f"f1: {n} connections x {L} B, 1 GPU" if world == 1 else f"f1: {n} connections/GPU",
                   "op": name + " (device mode)", "records_per_gpu": n, "record_bytes": L,
                   "frame_stride": FS if args.op == "rc4md5" else None,
                   "parallelism": f"connection-shard x{world}, no collective"},
        "roofline": {"bound": "hbm", "achieved": round(moved / step_s / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(moved / step_s / 1e9 / HBM_PEAK_GBS, 4),
                     **traffic_fields(args.pmc_summary, f"f1_{args.op}"),
                     "step_us_avg": round(step_s * 1e6, 2), "bytes_per_step": moved,
                     "compute": issue_compute(args.pmc_summary, f"f1_{args.op}", step_s,
                                              2 if args.op == "rc4md5" else 1),
                     "note": "algorithmic bytes read+written per step; the bound in practice is the per-byte "
                             "RC4 dependency chain through LDS (DESIGN.md)"},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.op == "rc4":
        th = cpu_threads()
        m = min(n, 16384)
        hst = st0[:m].copy()
        hd = host[: m * L].copy()
        ho = np.arange(m, dtype=np.uint64) * L
        hl = np.full(m, L, np.uint32)
        res = {}
        for t_ in (th, 1):
            mm = m if t_ > 1 else m // 16
            reps, t0 = 0, time.perf_counter()
            while time.perf_counter() - t0 < args.cpu_seconds / 2:
                oracle.rc4_crypt_batch(hst, hd, ho[:mm], hl[:mm], threads=t_)
                reps += 1
            res[t_] = (mm * L * reps / (time.perf_counter() - t0) / 2**30, reps, mm)
        gib, reps, mm = res[th]
        result["cpu_baseline"] = {"value": round(gib, 3), "unit": "GiB/s", "kind": "port", **core_counts(th, res[1][0]),
                                  "single_core_gib_s": round(res[1][0], 4),
                                  "sample": f"oracle BRB_RC4_Crypt restatement in place on {mm} connections x {L} B, "
                                            f"{reps} passes, {th} pthreads"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.op == "rc4md5":
        th = cpu_threads()
        m = min(n, 16384)
        hst = st0[:m].copy()
        ho = np.arange(m, dtype=np.uint64) * L
        hl = np.full(m, L, np.uint32)
        hfo = np.arange(m, dtype=np.uint64) * (L + H)
        hfl = np.full(m, L + H, np.uint32)
        hs = np.arange(m, dtype=np.uint64)
        hf = np.zeros(m * (L + H), np.uint8)
        hv = np.zeros(m, np.uint8)
        rs = st0[:m].copy()
        reps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < args.cpu_seconds:
            oracle.rc4md5_frame_batch(hst, host, ho, hl, hs, hf, hfo, threads=th)
            oracle.rc4md5_open_batch(rs, hf, hfo, hfl, hv, threads=th)
            reps += 1
        dt = time.perf_counter() - t0
        assert hv.all()
        result["cpu_baseline"] = {"value": round(m * L * reps / dt / 2**30, 3), "unit": "GiB/s", "cores": th,
                                  "nproc_note": "threads = the lease's CPU share (see the digest line's cores_note)",
                                  "kind": "port",
                                  "sample": f"oracle frame+open of {m} connections x {L} B, {reps} passes, {th} pthreads"}
    log(f"[bench] {name}: {step_s * 1e6:.1f} us per step")
    return result


def bench_var(args, rank, world, dev, stream, barrier, max_over_ranks, log):
    """BRB_MD5Batch / BrbSha1_Batch (byte offsets + lengths): 65 536 records per GPU with lengths
    uniform in [1000, 2000] bytes (1500 on average, the cfg2 volume) at arbitrary byte offsets
    (0..15-byte gaps), as a receive round hands over buffers of different sizes."""
    import numpy as np
    import torch

    import brb_framework_amd as brb
    from brb_framework_amd import workload

    n = args.records_per_gpu or 65536
    rng = np.random.default_rng(0x5EED0010 + rank)
    lens_h = rng.integers(1000, 2001, n).astype(np.uint32)
    if args.len_dist == "bimodal":        # diagnostic: 7 of 8 records 500 B, the others 8 000 B
        lens_h = np.where(rng.random(n) < 0.125, 8000, 500).astype(np.uint32)
    gaps = rng.integers(0, 16, n).astype(np.uint64)
    offs_h = np.cumsum(gaps + np.concatenate([[0], lens_h[:-1]]).astype(np.uint64)).astype(np.uint64)
    total = int(offs_h[-1] + lens_h[-1])
    host = workload.gen_records(workload.SEEDS[2], rank, 1, total + 16)
    n_rot = max(2, math.ceil(640e6 / host.nbytes))
    bufs = [torch.from_numpy(host).to(dev)]
    for _ in range(n_rot - 1):
        bufs.append(bufs[0].clone())
    width = 16 if args.op == "md5var" else 20
    offs = torch.from_numpy(offs_h.view(np.int64)).to(dev)
    lens = torch.from_numpy(lens_h.view(np.int32)).to(dev)
    out = torch.empty((n, width), dtype=torch.uint8, device=dev)
    Lb = brb.lib()
    cfn = Lb.BRB_MD5Batch if args.op == "md5var" else Lb.BrbSha1_Batch
    flags = brb.BATCH_DEVICE | brb.BATCH_ASYNC
    bptr = [b.data_ptr() for b in bufs]
    po, pl, pout = offs.data_ptr(), lens.data_ptr(), out.data_ptr()

    def launch(k, s, j=0):
        if cfn(bptr[k % n_rot], po, pl, n, pout, flags, s.cuda_stream) != 1:
            raise RuntimeError(Lb.BRB_CryptoGPU_LastError().decode())

    n_warm, n_steps = warm_up(args, launch, [stream], torch, max_over_ranks)
    wall, ev_s = timed_steps(lambda k, s, j: launch(k + n_warm, s, j), n_steps, [stream], barrier,
                             max_over_ranks, torch)
    got = out.cpu().numpy()
    h = hashlib.md5 if args.op == "md5var" else hashlib.sha1
    for i in list(rng.integers(0, n, 32)) + [0, n - 1]:
        o, L = int(offs_h[i]), int(lens_h[i])
        assert got[i].tobytes() == h(host[o:o + L].tobytes()).digest(), f"digest mismatch at {i}"
    step_s = ev_s
    payload = int(lens_h.sum())
    name = "BRB_MD5Batch" if args.op == "md5var" else "BrbSha1_Batch"
    result = {
        "metric": f"GiB/s of {'MD5' if args.op == 'md5var' else 'SHA-1'} over variable-length records "
                  "(offsets + lengths, 1000-2000 B)",
        "value": round(payload * world * n_steps / wall / 2**30, 2),
        "unit": "GiB/s", "n_gpus": world, "steps": n_steps, "warmup": n_warm,
        "ms_per_step": round(wall / n_steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u32",
        "data": f"synthetic (splitmix64 bytes, HBM-resident, {n_rot} rotating copies; lengths U[1000, 2000])",
        "config": {"workload": f"{n} records x 1000-2000 B at any byte offset" + (", 1 GPU" if world == 1 else "/GPU"),
                   "op": name + " (device mode)", "records_per_gpu": n, "record_bytes_mean": payload / n,
                   "parallelism": f"record-shard x{world}, no collective"},
        "roofline": {"bound": "hbm", "achieved": round(payload / step_s / 1e9, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(payload / step_s / 1e9 / HBM_PEAK_GBS, 4),
                     **traffic_fields(args.pmc_summary, f"var_{args.op}"),
                     "launch_us_avg": round(step_s * 1e6, 2), "bytes_per_launch": payload,
                     "compute": issue_compute(args.pmc_summary, f"var_{args.op}", step_s)},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import oracle     # test infrastructure: the CPU restatement is the baseline, never the product
        th = cpu_threads()
        fn = oracle.md5_batch if args.op == "md5var" else oracle.sha1_batch
        res = {}
        for t_ in (th, 1):
            m = n if t_ > 1 else n // 16
            fn(host, offs_h[:256], lens_h[:256], threads=t_)
            reps, t0 = 0, time.perf_counter()
            while True:
                dg = fn(host, offs_h[:m], lens_h[:m], threads=t_)
                reps += 1
                if time.perf_counter() - t0 >= args.cpu_seconds / 2:
                    break
            res[t_] = (int(lens_h[:m].sum()) * reps / (time.perf_counter() - t0) / 2**30, reps, m)
        assert np.array_equal(dg[:64], got[:64])
        gib, reps, m = res[th]
        result["cpu_baseline"] = {"value": round(gib, 3), "unit": "GiB/s", "kind": "port", **core_counts(th, res[1][0]),
                                  "single_core_gib_s": round(res[1][0], 4),
                                  "sample": f"oracle/brb_oracle.c {name} restatement over the same {m} records "
                                            f"(U[1000, 2000] B at their offsets), {reps} passes, {th} pthreads"}
        log(f"[bench] cpu baseline {gib:.2f} GiB/s on {th} threads")
    log(f"[bench] {name}: {step_s * 1e6:.1f} us per launch")
    return result


def bench_f4(args, rank, world, dev, stream, barrier, max_over_ranks, log):
    """SURVEY §8 f4 on the cfg2 shape (65 536 records of 1500 data bytes per GPU, HBM-resident).
    --op metadata: one step = BRB_MetaDataUnpackBatch over 65 536 MetaData packs of 4 items x 375 B
                   (1 664 bytes each: header, item headers, data, canaries), every pack valid.
    --op md5seg:   one step = BRB_MD5BatchSegments over the same packs' items (MetaDataHeaderLoadData,
                   meta_data.c:397-433: MD5 of a MetaData's 4 item ranges), checked against the
                   digests the packs carry.
    --op base64:   one step = BRB_Base64EncodeBatch of the 1500-byte records (2000 characters each),
                   then BRB_Base64DecodeBatch of those texts back into 1500-byte records."""
    import numpy as np
    import torch

    import brb_framework_amd as brb
    from brb_framework_amd import workload
    import oracle

    L = 1500
    n = args.records_per_gpu or 65536
    host = workload.gen_records(workload.SEEDS[2], rank * n, n, L)
    Lb = brb.lib()
    flags = brb.BATCH_DEVICE | brb.BATCH_ASYNC
    if args.op in ("metadata", "md5seg"):
        K, Q = 4, L // 4                         # items per pack, bytes per item
        P_SZ = 64 + K * (24 + Q + 1)
        packs = np.zeros((n, P_SZ), np.uint8)
        hdr = np.zeros(64, np.uint8)
        hdr[:24] = np.frombuffer(np.array([0, K], "<i4").tobytes() + np.array([P_SZ - 64], "<u8").tobytes()
                                 + b"BRB_META", np.uint8)
        packs[:, :64] = hdr
        packs[:, 24:40] = brb.md5_batch_fixed(host, L, n)        # MD5 of the items' concatenation
        for j in range(K):
            o = 64 + j * (24 + Q + 1)
            packs[:, o:o + 24] = np.frombuffer(np.array([j + 1, 0, Q], "<u8").tobytes(), np.uint8)
            packs[:, o + 24:o + 24 + Q] = host.reshape(n, L)[:, j * Q:(j + 1) * Q]
            packs[:, o + 24 + Q] = 0x1F
        flat = packs.reshape(-1)
        offs_h = np.arange(n, dtype=np.uint64) * P_SZ
        lens_h = np.full(n, P_SZ, np.uint32)
        n_rot = max(2, math.ceil(640e6 / flat.nbytes))
        bufs = [torch.from_numpy(flat).to(dev)]
        for _ in range(n_rot - 1):
            bufs.append(bufs[0].clone())
        offs = torch.from_numpy(offs_h.view(np.int64)).to(dev)
        lens = torch.from_numpy(lens_h.view(np.int32)).to(dev)
        info = torch.zeros((n, 32), dtype=torch.uint8, device=dev)
        bptr = [b.data_ptr() for b in bufs]
        po, pl, pi = offs.data_ptr(), lens.data_ptr(), info.data_ptr()

        if args.op == "metadata":
            def launch(k, s, j=0):
                if Lb.BRB_MetaDataUnpackBatch(bptr[k % n_rot], po, pl, n, pi, flags, s.cuda_stream) != 1:
                    raise RuntimeError(Lb.BRB_CryptoGPU_LastError().decode())
            moved, payload, name = n * (P_SZ + 32), n * P_SZ, "BRB_MetaDataUnpackBatch"
            metric = "GiB/s of MetaData packs validated (MetaDataUnpack: walk, canaries, MD5) (SURVEY §8 f4)"
        else:
            item0 = np.array([64 + j * (24 + Q + 1) + 24 for j in range(K)], np.uint64)
            soffs = torch.from_numpy((offs_h[:, None] + item0[None, :]).reshape(-1).view(np.int64)).to(dev)
            slens = torch.full((n * K,), Q, dtype=torch.int32, device=dev)
            sfirst = torch.from_numpy((np.arange(n + 1, dtype=np.uint64) * K).view(np.int64)).to(dev)
            digs = torch.zeros((n, 16), dtype=torch.uint8, device=dev)
            so, sl, sf, pd = soffs.data_ptr(), slens.data_ptr(), sfirst.data_ptr(), digs.data_ptr()

            def launch(k, s, j=0):
                if Lb.BRB_MD5BatchSegments(bptr[k % n_rot], so, sl, sf, n, pd, flags, s.cuda_stream) != 1:
                    raise RuntimeError(Lb.BRB_CryptoGPU_LastError().decode())
            moved, payload, name = n * (K * Q + 16), n * K * Q, "BRB_MD5BatchSegments"
            metric = "GiB/s of MetaData item bytes digested (MetaDataHeaderLoadData: MD5 over a record's segments) (SURVEY §8 f4)"
    else:
        T = 4 * ((L + 2) // 3)
        n_rot = max(2, math.ceil(640e6 / host.nbytes))
        bufs = [torch.from_numpy(host).to(dev)]
        for _ in range(n_rot - 1):
            bufs.append(bufs[0].clone())
        offs = torch.from_numpy((np.arange(n, dtype=np.uint64) * L).view(np.int64)).to(dev)
        lens = torch.full((n,), L, dtype=torch.int32, device=dev)
        toffs = torch.from_numpy((np.arange(n, dtype=np.uint64) * T).view(np.int64)).to(dev)
        tlens = torch.full((n,), T, dtype=torch.int32, device=dev)
        text = torch.zeros(n * T, dtype=torch.uint8, device=dev)
        back = torch.zeros(n * L, dtype=torch.uint8, device=dev)
        olens = torch.zeros(n, dtype=torch.int32, device=dev)
        bptr = [b.data_ptr() for b in bufs]
        P = [x.data_ptr() for x in (offs, lens, toffs, tlens, text, back, olens)]

        def launch(k, s, j=0):
            h = s.cuda_stream
            rc = Lb.BRB_Base64EncodeBatch(bptr[k % n_rot], P[0], P[1], n, P[4], P[2], flags, h)
            if rc == 1:
                rc = Lb.BRB_Base64DecodeBatch(P[4], P[2], P[3], n, P[5], P[0], P[6], flags, h)
            if rc != 1:
                raise RuntimeError(Lb.BRB_CryptoGPU_LastError().decode())
        moved, payload, name = n * (2 * L + 2 * T + 4), n * L, "BRB_Base64EncodeBatch + BRB_Base64DecodeBatch"
        metric = "GiB/s of records per base64 encode + decode round trip (SURVEY §8 f4)"

    n_warm, n_steps = warm_up(args, launch, [stream], torch, max_over_ranks)
    wall, ev_s = timed_steps(lambda k, s, j: launch(k + n_warm, s, j), n_steps, [stream], barrier,
                             max_over_ranks, torch)
    torch.cuda.synchronize()
    if args.op == "metadata":
        got = info.cpu().numpy().reshape(-1).view(brb.METADATA_INFO_DTYPE)
        assert (got["error_code"] == 7).all() and (got["item_count"] == 4).all(), "a pack failed to unpack"
        assert (got["cur_offset"] == P_SZ).all()
    elif args.op == "md5seg":
        assert np.array_equal(digs.cpu().numpy(), packs[:, 24:40]), "segment digests differ from the packs' digests"
    else:
        assert (olens.cpu().numpy() == L).all()
        last = (n_warm + n_steps - 1) % n_rot
        assert torch.equal(back, bufs[last]), "base64 round trip changed the records"
    step_s = ev_s
    result = {
        "metric": metric,
        "value": round(payload * world * n_steps / wall / 2**30, 2),
        "unit": "GiB/s", "n_gpus": world, "steps": n_steps, "warmup": n_warm,
        "ms_per_step": round(wall / n_steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8",
        "data": f"synthetic (splitmix64 records, HBM-resident, {n_rot} rotating copies)",
        "config": {"workload": f"f4 {args.op}: {n} records x {L} data bytes" + (", 1 GPU" if world == 1 else "/GPU"),
                   "op": name + " (device mode)", "records_per_gpu": n, "record_bytes": L,
                   "parallelism": f"record-shard x{world}, no collective"},
        "roofline": {"bound": "hbm", "achieved": round(moved / step_s / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(moved / step_s / 1e9 / HBM_PEAK_GBS, 4),
                     **traffic_fields(args.pmc_summary, f"f4_{args.op}"),
                     "step_us_avg": round(step_s * 1e6, 2), "bytes_per_step": moved,
                     "compute": (issue_compute(args.pmc_summary, f"f4_{args.op}", step_s,
                                               2 if args.op == "base64" else 1)),
                     "note": ("algorithmic bytes read + written per step; base64: 32 lanes per record, 12/16-byte "
                              "pieces, 8 waves per SIMD (HBM-bound, DESIGN.md 4.5)" if args.op == "base64" else
                              "algorithmic bytes read + written per step; one lane per record, so the bound in "
                              "practice is per-lane issue (MD5 for metadata), DESIGN.md")},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        th = cpu_threads()
        m = min(n, 16384)
        reps, t0 = 0, time.perf_counter()
        if args.op == "md5seg":
            # the same digests on the CPU: the oracle's MD5 over each record's items, which are the
            # record's 1500 bytes back to back
            while time.perf_counter() - t0 < args.cpu_seconds:
                dg = oracle.md5_batch_fixed(host[: m * L], L, m, threads=th)
                reps += 1
            assert np.array_equal(dg, packs[:m, 24:40])
            cores, sample = th, f"oracle MD5 of {m} records' 4 x {Q} B items (concatenated), {reps} passes, {th} pthreads"
        elif args.op == "metadata":
            fl = flat[: m * P_SZ]
            while time.perf_counter() - t0 < args.cpu_seconds:
                inf = oracle.metadata_unpack_batch(fl, offs_h[:m], lens_h[:m], threads=th)
                reps += 1
            assert (inf.view("<i4")[:, 0] == 7).all()
            cores, sample = th, f"oracle MetaDataUnpack of {m} packs x {P_SZ} B, {reps} passes, {th} pthreads"
        else:
            m = min(n, 2048)
            recs = [host[i * L:(i + 1) * L].tobytes() for i in range(m)]
            while time.perf_counter() - t0 < args.cpu_seconds:
                for r in recs:
                    assert oracle.b64_decode(oracle.b64_encode(r)) == r
                reps += 1
            cores, sample = 1, f"oracle encode + decode of {m} records x {L} B, {reps} passes, 1 thread"
        dt = time.perf_counter() - t0
        result["cpu_baseline"] = {"value": round(m * L * reps / dt / 2**30, 3) if args.op in ("base64", "md5seg")
                                  else round(m * P_SZ * reps / dt / 2**30, 3), "unit": "GiB/s", "cores": cores,
                                  "kind": "port", "sample": sample}
    log(f"[bench] {name}: {step_s * 1e6:.1f} us per step")
    return result


# ------------------------------------------------------------------------------------------------
def bench_batcher(args, rank, world, log):
    """SURVEY §8 f2, host-inclusive: one event-loop round = C connections each receiving one
    1500-byte RC4+MD5 frame and sending one 1500-byte payload, driven from C the way an event loop
    would (tools/batcher_bench.c: one BRB_TransformBatcherRead/Write call per buffer, one Flush per
    round).  Run as a child process (it opens the GPU itself)."""
    exe = os.path.join(ROOT, "tools", "batcher_bench")
    src = exe + ".c"
    lib = os.path.join(ROOT, "brb_framework_amd")
    if not os.path.exists(exe) or os.path.getmtime(exe) < os.path.getmtime(src):
        subprocess.run(["gcc", "-O2", "-pthread", "-I", os.path.join(ROOT, "include"), src, "-L", lib, "-lbrb_crypto_gpu",
                        f"-Wl,-rpath,{lib}", "-o", exe], check=True)
    C = args.records_per_gpu or 16384
    steps = 20 if args.steps is None else args.steps
    warm = 20 if args.warmup is None else args.warmup
    def run(zc, pipelined=0, threads=1):
        out = subprocess.run([exe, str(C), "1500", str(steps), str(warm), str(zc), str(pipelined), str(threads)],
                             check=True,
                             capture_output=True,
                             text=True, timeout=600).stdout
        r = json.loads(out.strip().splitlines()[-1])
        if "error" in r:
            raise SystemExit("batcher_bench: " + r["error"])
        return r
    r, z, rp, zp, rp4 = run(0), run(1), run(0, 1), run(1, 1), run(0, 1, 4)
    t = r["round_ms_mean"] / 1e3
    return {"metric": "GiB/s of payload through the receive-loop transform batcher (SURVEY §8 f2, host-inclusive)",
            "value": r["payload_gib_s"], "unit": "GiB/s", "n_gpus": world, "steps": steps,
            "warmup": warm, "ms_per_step": round(t * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (peer frames built with the compat BRB_RC4/BRB_MD5 calls outside the timed region)",
            "config": {"workload": f"f2: {C} connections x (1 frame in + 1 payload out) x 1500 B per round",
                       "op": "tools/batcher_bench.c: BRB_TransformBatcherRead/Write per buffer + Flush per round",
                       "parallelism": "single GPU"},
            "buffers_per_s": r["buffers_per_s"], "round_ms_min": r["round_ms_min"],
            "submit_ms_median": r["submit_ms_median"],
            "zero_copy": {"value": z["payload_gib_s"], "unit": "GiB/s", "ms_per_step": z["round_ms_mean"],
                          "submit_ms_median": z["submit_ms_median"],
                          "op": "BRB_BATCHER_ZERO_COPY: buffers page-locked once (BRB_CryptoGPU_HostRegister), "
                                "kernels read them and write results over PCIe, no arena copies"},
            "pipelined": {"copy": {"value": rp["payload_gib_s"], "ms_per_step": rp["round_ms_mean"],
                                   "submit_ms_median": rp["submit_ms_median"]},
                          "zero_copy": {"value": zp["payload_gib_s"], "ms_per_step": zp["round_ms_mean"],
                                        "submit_ms_median": zp["submit_ms_median"]},
                          "copy_4_submit_threads": {"value": rp4["payload_gib_s"], "ms_per_step": rp4["round_ms_mean"],
                                                    "submit_ms_median": rp4["submit_ms_median"]},
                          "unit": "GiB/s",
                          "op": "BRB_BATCHER_PIPELINED: FlushAsync per round, the loop submits round k+1 while "
                                "the GPU runs round k"},
            "note": "step = one round: per-buffer submit (copy into the pinned arena), H2D, open + frame kernels, "
                    "D2H, one callback per buffer"}


if __name__ == "__main__":
    main()
