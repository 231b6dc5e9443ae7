#!/bin/bash
# Session check: parity tests + digest benches (gpu_s3.sh), the <= 64 B A/B sweep, RC4 benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-s3e}
O=gpurun_out/$T
bash tools/gpu_s3.sh "$T" || exit 1
timeout -k 10 120 tools/mb/md5ab 1048576 64 > $O/ab3.txt 2>&1 || exit 1
cat $O/ab3.txt
for op in rc4 rc4md5; do
  timeout -k 10 200 python bench.py --op $op --no-cpu-baseline > $O/$op.json 2> $O/$op.err || { cat $O/$op.err; exit 1; }
  cat $O/$op.json
done
