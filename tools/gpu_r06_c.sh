#!/bin/bash
# Round 6: segment / MetaData parity with the no-wrap emission (in-tree build), RC4 parity of the
# early-S[j] generator build (gpurun_tmp_libs/c_*.so swapped in), then interleaved A/B of every
# build under gpurun_tmp_libs/ on rc4, rc4md5, md5seg and metadata.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06c}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_segments.py tests/test_metadata.py \
    > $O/pytest_seg.log 2>&1 || { tail -40 $O/pytest_seg.log; exit 1; }
tail -1 $O/pytest_seg.log
cp brb_framework_amd/libbrb_crypto_gpu.so $O/intree.so
cp gpurun_tmp_libs/c_rc4jearly.so brb_framework_amd/libbrb_crypto_gpu.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_rc4.py tests/test_batcher.py \
    > $O/pytest_rc4je.log 2>&1; rc=$?; cp $O/intree.so brb_framework_amd/libbrb_crypto_gpu.so
tail -1 $O/pytest_rc4je.log; [ $rc -eq 0 ] || { tail -30 $O/pytest_rc4je.log; exit 1; }
bash tools/gpu_ab_libs.sh ${1:-r06c}/ab_rc4 ${R:-3} --op rc4 && bash tools/gpu_ab_libs.sh ${1:-r06c}/ab_rc4md5 ${R:-3} --op rc4md5 &&
bash tools/gpu_ab_libs.sh ${1:-r06c}/ab_md5seg ${R:-3} --op md5seg && bash tools/gpu_ab_libs.sh ${1:-r06c}/ab_metadata ${R:-3} --op metadata
