#!/bin/bash
# Round 3: the cause of round 2's all-zero batcher state, then the GPU suite and the
# default bench.  The two regression tests run first against the round-2 library
# (gpurun_tmp_libs/old_r02.so, expected to FAIL if Create's default-stream hipMemset is the cause),
# then everything against the in-tree build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03a}; mkdir -p $O
cp brb_framework_amd/libbrb_crypto_gpu.so $O/new.so
cp gpurun_tmp_libs/old_r02.so brb_framework_amd/libbrb_crypto_gpu.so
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_batcher.py -m gpu \
    -k "busy_default_stream or after_rc4" > $O/old_lib.log 2>&1
echo "round-2 library: pytest rc=$?"
grep -E "PASSED|FAILED|Error" $O/old_lib.log | head -20
cp $O/new.so brb_framework_amd/libbrb_crypto_gpu.so
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
