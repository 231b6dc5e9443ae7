#!/bin/bash
# Session check: batcher tests (copy + zero-copy), then the batcher bench in both modes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-zc}; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_batcher.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -12 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for zc in 0 1; do
  timeout -k 10 120 tools/batcher_bench 16384 1500 20 5 $zc > $O/bb$zc.json 2>&1 || { cat $O/bb$zc.json; exit 1; }
  cat $O/bb$zc.json
done
timeout -k 10 120 tools/batcher_bench 4096 1500 20 5 1 && timeout -k 10 120 tools/batcher_bench 65536 1500 10 3 1
