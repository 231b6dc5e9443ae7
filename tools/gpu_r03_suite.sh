#!/bin/bash
# The whole -m gpu suite (one process, per-test time limit), then the variable-length A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03s}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1
rc=$?; grep -E "FAILED|Error" $O/gpu_tests.log | head -5; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
[ "${2:-}" = "novar" ] || bash tools/gpu_r03_var.sh "${1:-r03s}_var" notests 2>&1 | grep -v PASSED
