#!/bin/bash
# Batcher tests, then both round modes and the zero-copy kernel times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-zc4}; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_batcher.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tools/batcher_bench 16384 1500 20 5 1 || exit 1
timeout -k 10 120 tools/batcher_bench 16384 1500 20 5 0 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- tools/batcher_bench 16384 1500 20 5 1 > $O/bbp.json 2>&1 || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('$O/p/run_kernel_stats.csv')): print(r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3)"
