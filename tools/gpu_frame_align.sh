#!/bin/bash
# does the RC4+MD5 frame/open write amplification cost time or only bytes?
# The same kernels on frames packed back to back (1530-byte stride: every frame's payload starts at
# a 4-byte phase inside its sectors) and on 64-byte-aligned frames (1536-byte stride), interleaved,
# then one WRITE_SIZE/FETCH_SIZE pass for each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-fa}
O=gpurun_out/$T
mkdir -p $O
for r in ${ROUNDS:-3}; do
  for fs in 1530 1536; do
    timeout -k 10 200 python3 bench.py --op rc4md5 --frame-stride $fs --no-cpu-baseline > $O/fs-$fs-$r.json 2> $O/fs-$fs-$r.err || { tail -3 $O/fs-$fs-$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/fs-$fs-$r.json')); print('stride $fs', $r, d['value'], d['roofline']['step_us_avg'])"
  done
done
for fs in 1530 1536; do
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$O/pmc$fs" -o run -- \
      python3 bench.py --op rc4md5 --frame-stride $fs --no-cpu-baseline --steps 10 --warmup 2 > "$O/pmc$fs.log" 2>&1 || { echo "pmc failed"; exit 1; }
  python3 tools/pmc_summary.py "$O/pmc$fs" rc4 | grep -E "WRITE|kernel_us"
done
echo done
