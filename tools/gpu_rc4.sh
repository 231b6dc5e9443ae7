#!/bin/bash
# RC4 check: RC4 / batcher GPU tests, then the f1 benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-rc4}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_rc4.py tests/test_batcher.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for op in rc4 rc4md5; do
  timeout -k 10 200 python bench.py --op $op --no-cpu-baseline > $O/$op.json 2> $O/$op.err || { cat $O/$op.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$op.json')); r=d['roofline']; print('$op', d['value'], d['unit'], 'step_us', r['step_us_avg'])"
done
