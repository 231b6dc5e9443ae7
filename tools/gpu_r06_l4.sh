#!/bin/bash
# Round 6 experiment: the half-line line kernel (tools/mb/line4_kernel.h, four waves per SIMD)
# against the product's -- parity over several record lengths, then the A/B on the cfg5 shard and cfg2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r06l4}
mkdir -p $O
for L in 68 100 132 1000 1500 1504 1536 1540 4096; do
    timeout -k 10 60 tools/mb/line_ab 65600 $L 1 20 > $O/parity_$L.txt 2>&1 || { tail -5 $O/parity_$L.txt; exit 1; }
    head -1 $O/parity_$L.txt
done
timeout -k 10 300 tools/mb/line_ab 1048576 1500 ${ROUNDS:-5} 40 > $O/line_ab_cfg5.txt 2>&1 || { tail -5 $O/line_ab_cfg5.txt; exit 1; }
grep -E "^n=|MEDIAN" $O/line_ab_cfg5.txt
timeout -k 10 200 tools/mb/line_ab 65536 1500 ${ROUNDS:-5} 400 > $O/line_ab_cfg2.txt 2>&1 || { tail -5 $O/line_ab_cfg2.txt; exit 1; }
grep -E "^n=|MEDIAN" $O/line_ab_cfg2.txt
