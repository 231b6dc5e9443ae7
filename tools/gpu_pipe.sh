#!/bin/bash
# Batcher rounds: parity (test_batcher.py, every mode) then the host-inclusive bench in each mode
# (copy / zero-copy x one round at a time / pipelined x submit threads).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pipe}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_batcher.py -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 && echo "pytest ok" &&
for m in "0 0 1" "0 1 1" "1 0 1" "1 1 1" "0 0 4" "0 1 4" "0 1 8" "1 0 4" "1 1 4"; do
  set -- $m
  f="$OUT/bb_zc$1_p$2_t$3.json"
  timeout -k 10 180 tools/batcher_bench 16384 1500 20 20 $1 $2 $3 > "$f" 2>&1 || { cat "$f"; exit 1; }
  cat "$f"
done
rc=$?
tail -4 "$OUT/pytest.log"
exit $rc
