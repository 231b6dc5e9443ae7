#!/bin/bash
# Round 6 experiment: the cfg5 shard's groups split over the XCDs by weight from per-XCD end-time
# feedback (tools/mb/line_xcd.hip), against the product kernel, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r06xcd}
mkdir -p $O
timeout -k 10 300 tools/mb/line_xcd 1048576 1500 ${ROUNDS:-5} 40 > $O/line_xcd_cfg5.txt 2>&1 || { tail -5 $O/line_xcd_cfg5.txt; exit 1; }
cat $O/line_xcd_cfg5.txt
