#!/bin/bash
# Session check: all GPU tests, cfg2/cfg5 A/B of the digest kernels, default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-s3f}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tools/mb/md5ab 65536 1500 > $O/ab2.txt 2>&1 || exit 1
timeout -k 10 120 tools/mb/md5ab 1048576 1500 > $O/ab5.txt 2>&1 || exit 1
cat $O/ab2.txt $O/ab5.txt
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b2.json 2> $O/b2.err || exit 1
cat $O/b2.json
