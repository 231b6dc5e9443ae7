#!/bin/bash
# Round 6: the batcher's key-epoch poisoning, the async fault word's cleanup, and the
# line kernel again (prologue order fixed): parity, then line_ab on cfg5 and cfg2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06b}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_batcher.py tests/test_gpu_parity.py tests/test_rc4.py \
    -k "${SEL:-batcher or fault or async or line_kernel or cfg5_full or cfg2_full or large_batch or many_groups}" \
    > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 tools/mb/line_ab 1048576 1500 ${ROUNDS:-5} 40 > $O/line_ab_cfg5.txt 2>&1 || { tail -5 $O/line_ab_cfg5.txt; exit 1; }
grep -E "^n=|MEDIAN" $O/line_ab_cfg5.txt
timeout -k 10 200 tools/mb/line_ab 65536 1500 ${ROUNDS:-5} 400 > $O/line_ab_cfg2.txt 2>&1 || { tail -5 $O/line_ab_cfg2.txt; exit 1; }
grep -E "^n=|MEDIAN" $O/line_ab_cfg2.txt
