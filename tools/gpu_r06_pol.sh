#!/bin/bash
# Round 6 experiment: cache policy of the line kernel's streamed DMAs (tools/mb/line_pol.hip),
# cfg5 shard and cfg2, interleaved, digests compared first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r06pol}
mkdir -p $O
timeout -k 10 400 tools/mb/line_pol 1048576 1500 ${ROUNDS:-4} 30 > $O/line_pol_cfg5.txt 2>&1 || { tail -5 $O/line_pol_cfg5.txt; exit 1; }
grep -E "^n=|MEDIAN" $O/line_pol_cfg5.txt
timeout -k 10 200 tools/mb/line_pol 65536 1500 ${ROUNDS:-4} 300 > $O/line_pol_cfg2.txt 2>&1 || { tail -5 $O/line_pol_cfg2.txt; exit 1; }
grep -E "^n=|MEDIAN" $O/line_pol_cfg2.txt
