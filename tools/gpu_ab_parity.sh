#!/bin/bash
# Parity of every library build under gpurun_tmp_libs/*.so: runs the given -m gpu test files once
# per build (the build copied in-tree first); the first failure ends the call.  The in-tree library
# is restored at the end.
#   tools/gpu_ab_parity.sh <tag> <test files...>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-abt}; shift
mkdir -p $O
cp brb_framework_amd/libbrb_crypto_gpu.so $O/intree.so
rc=0
for v in gpurun_tmp_libs/*.so; do
  n=$(basename $v .so)
  cp $v brb_framework_amd/libbrb_crypto_gpu.so
  timeout -k 10 600 python3 -u -m pytest "$@" -m gpu -x -q --timeout 200 --timeout-method thread > $O/$n.log 2>&1 \
    && echo "$n parity ok: $(tail -1 $O/$n.log)" || { echo "$n parity FAILED"; tail -15 $O/$n.log; rc=1; break; }
done
cp $O/intree.so brb_framework_amd/libbrb_crypto_gpu.so
exit $rc
