#!/bin/bash
# Round 6: the product line kernel with its DMA compiled out (BRB_LINE_NO_DMA: hashes stale LDS),
# per-wave stamps -- the compression's issue rate and clock without the memory side.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r06nodma}
mkdir -p $O
timeout -k 10 200 tools/mb/line_probe6_nodma 65536 1500 r06 > $O/nodma_cfg2.txt 2>&1 || { tail -5 $O/nodma_cfg2.txt; exit 1; }
cat $O/nodma_cfg2.txt
timeout -k 10 200 tools/mb/line_probe6_nodma 1048576 1500 r06 > $O/nodma_cfg5.txt 2>&1 || { tail -5 $O/nodma_cfg5.txt; exit 1; }
cat $O/nodma_cfg5.txt
timeout -k 10 200 tools/mb/line_probe6 65536 1500 r06 > $O/dma_cfg2.txt 2>&1 || { tail -5 $O/dma_cfg2.txt; exit 1; }
grep -E "per-XCC|span" $O/dma_cfg2.txt
