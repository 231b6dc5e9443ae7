#!/bin/bash
# Variable-length bucketing: parity (every var-length test) and the md5var / sha1var bench lines
# with bucketing on and off (test option var_sort), interleaved, one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03var}; mkdir -p $O
if [ "${2:-}" != "notests" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu \
      -k "variable" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2; do
  for n in 65536 524288; do
    for op in md5var sha1var; do
      for v in 1 0; do
        timeout -k 10 200 python3 bench.py --op $op --records-per-gpu $n --no-cpu-baseline --test-option var_sort=$v > $O/$op-$n-$v-$r.json 2> $O/$op-$n-$v-$r.err || { tail -3 $O/$op-$n-$v-$r.err; exit 1; }
        python3 -c "import json; d=json.load(open('$O/$op-$n-$v-$r.json')); print('$op n=$n var_sort=$v', $r, d['value'], d['roofline']['launch_us_avg'], d['roofline']['frac'])"
      done
    done
  done
done
