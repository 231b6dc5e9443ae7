#!/bin/bash
# Session check: all GPU tests, RC4 part timings, f1 benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-s3h}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tools/mb/rc4parts > $O/parts.txt 2>&1 || exit 1
cat $O/parts.txt
for op in rc4 rc4md5; do
  timeout -k 10 200 python bench.py --op $op --no-cpu-baseline > $O/$op.json 2> $O/$op.err || { cat $O/$op.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$op.json')); r=d['roofline']; print('$op', d['value'], d['unit'], 'step_us', r['step_us_avg'])"
done
