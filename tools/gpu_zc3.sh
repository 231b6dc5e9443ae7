#!/bin/bash
# Kernel times of the batcher rounds (copy / zero-copy) under rocprofv3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-zc3}; mkdir -p $O
for zc in 0 1; do
  timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/p$zc -o run -- tools/batcher_bench 16384 1500 20 5 $zc > $O/bb$zc.json 2>&1 || { tail -5 $O/bb$zc.json; exit 1; }
  tail -1 $O/bb$zc.json
done
find $O -name "*stats.csv" | sort | while read f; do echo "== $f"; cut -d, -f1-8 "$f" | head -8; done
