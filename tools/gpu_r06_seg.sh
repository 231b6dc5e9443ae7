#!/bin/bash
# Round 6: emission without the ring's wrap mask when no lane wraps -- the
# segment and MetaData parity suites, then an interleaved A/B of the builds under gpurun_tmp_libs/
# on --op md5seg and --op metadata.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06seg}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_segments.py tests/test_metadata.py \
    > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu_ab_libs.sh ${1:-r06seg}/ab_md5seg ${R:-3} --op md5seg && bash tools/gpu_ab_libs.sh ${1:-r06seg}/ab_metadata ${R:-3} --op metadata
