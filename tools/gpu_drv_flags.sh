#!/bin/bash
# bench.py's own 20-step region in isolation (tools/mb/short_region2.py), then the headline at the
# driver's flags three times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/${1:-drv} && timeout -k 10 300 python -u tools/mb/short_region2.py 12 > gpurun_out/${1:-drv}/sr2.txt 2>&1 && for i in 1 2 3; do timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${1:-drv}/n1_$i.json 2> gpurun_out/${1:-drv}/n1_$i.err || exit 1; done; echo ok
