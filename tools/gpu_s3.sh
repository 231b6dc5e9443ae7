#!/bin/bash
# Session check: GPU parity tests, then short benches of the digest configs (no CPU baseline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-s3}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for c in "--config 2" "--config 2 --op sha1" "--config 3" "--config 5" $EXTRA; do
  tag=$(echo $c | tr -d ' -')
  timeout -k 10 200 python bench.py $c --no-cpu-baseline --no-pcie > $O/$tag.json 2> $O/$tag.err || { cat $O/$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); r=d['roofline']; print('$c', d['value'], d['unit'], d.get('mrecords_per_s'), 'kern_us', r.get('launch_us_avg'), 'frac', r['frac'])"
done
