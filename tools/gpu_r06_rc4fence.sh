#!/bin/bash
# Round 6: the RC4 step with sched_barrier fences (rc4_device.h) -- RC4 / batcher parity suites, then
# an interleaved A/B of the library builds under gpurun_tmp_libs/ on the RC4 pass and the RC4+MD5
# frame / open line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06rc4f}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_rc4.py tests/test_batcher.py \
    > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu_ab_libs.sh ${1:-r06rc4f}/ab_rc4 ${R:-3} --op rc4 && bash tools/gpu_ab_libs.sh ${1:-r06rc4f}/ab_rc4md5 ${R:-3} --op rc4md5
