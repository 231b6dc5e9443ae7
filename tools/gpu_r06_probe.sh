#!/bin/bash
# Round 6: per-wave stamps of the product line kernel (tools/mb/line_probe.hip "r06" mode): the
# in-kernel clock, start / end spread, DMA wait fraction -- cfg5 shard and cfg2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r06probe}
mkdir -p $O
timeout -k 10 200 tools/mb/line_probe6 1048576 1500 r06 > $O/probe_cfg5.txt 2>&1 || { tail -5 $O/probe_cfg5.txt; exit 1; }
cat $O/probe_cfg5.txt
timeout -k 10 200 tools/mb/line_probe6 65536 1500 r06 > $O/probe_cfg2.txt 2>&1 || { tail -5 $O/probe_cfg2.txt; exit 1; }
cat $O/probe_cfg2.txt
