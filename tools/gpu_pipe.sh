#!/bin/bash
# Pipelined batcher rounds: parity (test_batcher.py, every mode) then the host-inclusive bench in
# the four modes (copy / zero-copy x one round at a time / pipelined).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pipe}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_batcher.py -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 && echo "pytest ok" &&
for m in "0 0" "0 1" "1 0" "1 1"; do
  set -- $m
  timeout -k 10 180 tools/batcher_bench 16384 1500 20 20 $1 $2 > "$OUT/bb_zc$1_p$2.json" 2>&1 || { cat "$OUT/bb_zc$1_p$2.json"; exit 1; }
  cat "$OUT/bb_zc$1_p$2.json"
done
rc=$?
tail -4 "$OUT/pytest.log"
exit $rc
