#!/bin/bash
# RC4-family check: RC4 / batcher parity tests, then the rc4 and rc4md5 bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-rc4w}; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_rc4.py tests/test_batcher.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for op in rc4 rc4md5; do
  timeout -k 10 200 python bench.py --op $op --no-cpu-baseline > $O/$op.json 2> $O/$op.err || { cat $O/$op.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$op.json')); r=d['roofline']; print('$op', d['value'], d['unit'], 'step_us', r.get('step_us_avg'), r.get('launch_us_avg'))"
done
timeout -k 10 120 tools/batcher_bench 16384 1500 20 5 0 && timeout -k 10 120 tools/batcher_bench 16384 1500 20 5 1
