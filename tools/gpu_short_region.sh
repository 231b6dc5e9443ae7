#!/bin/bash
# tools/mb/short_region.py with HIP's default scheduling and with hipDeviceScheduleSpin, then
# bench.py's own warm-up + 20-step region repeated (tools/mb/short_region2.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-shortreg}
mkdir -p "$OUT"
timeout -k 10 180 python -u tools/mb/short_region.py > "$OUT/default.txt" 2>&1 && cat "$OUT/default.txt" &&
timeout -k 10 180 python -u tools/mb/short_region.py --spin > "$OUT/spin.txt" 2>&1 && cat "$OUT/spin.txt" &&
timeout -k 10 300 python -u tools/mb/short_region2.py 12 > "$OUT/bench_region.txt" 2>&1 && cat "$OUT/bench_region.txt"
