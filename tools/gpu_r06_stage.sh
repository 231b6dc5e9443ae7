#!/bin/bash
# Round 6 experiment: window-read placement in the line kernel (tools/mb/line_stage.hip), cfg2 and
# the cfg5 shard, interleaved, digests compared first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r06stage}
mkdir -p $O
timeout -k 10 200 tools/mb/line_stage 65536 1500 ${ROUNDS:-6} 300 > $O/line_stage_cfg2.txt 2>&1 || { tail -5 $O/line_stage_cfg2.txt; exit 1; }
grep -E "^n=|MEDIAN" $O/line_stage_cfg2.txt
timeout -k 10 300 tools/mb/line_stage 1048576 1500 ${ROUNDS:-4} 30 > $O/line_stage_cfg5.txt 2>&1 || { tail -5 $O/line_stage_cfg5.txt; exit 1; }
grep -E "^n=|MEDIAN" $O/line_stage_cfg5.txt
