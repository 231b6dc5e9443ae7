#!/bin/bash
# Round 6: per-SIMD ticket counters (digest_line_kernel<..., SCHED = 1>) against the per-workgroup
# counter, in-process (tools/mb/line_ab: round 5's form, round 6's, round 6's with per-SIMD tickets).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06e}
mkdir -p $O
timeout -k 10 300 tools/mb/line_ab 1048576 1500 5 40 > $O/line_ab_cfg5.txt 2>&1 || { tail -5 $O/line_ab_cfg5.txt; exit 1; }
grep -E "^n=|MEDIAN" $O/line_ab_cfg5.txt
timeout -k 10 200 tools/mb/line_ab 65536 1500 5 400 > $O/line_ab_cfg2.txt 2>&1 || { tail -5 $O/line_ab_cfg2.txt; exit 1; }
grep -E "^n=|MEDIAN" $O/line_ab_cfg2.txt
timeout -k 10 300 tools/mb/line_ab 300001 1500 5 100 > $O/line_ab_300k.txt 2>&1 || { tail -5 $O/line_ab_300k.txt; exit 1; }
grep -E "^n=|MEDIAN" $O/line_ab_300k.txt
