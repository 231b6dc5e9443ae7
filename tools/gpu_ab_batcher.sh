#!/bin/bash
# Interleaved A/B of library builds (gpurun_tmp_libs/) on the batcher benchmark, copy mode.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-abbat}; mkdir -p $O
cp brb_framework_amd/libbrb_crypto_gpu.so $O/orig.so
for r in 1 2 3; do
  for v in gpurun_tmp_libs/*.so; do
    cp $v brb_framework_amd/libbrb_crypto_gpu.so
    echo -n "$(basename $v .so) $r "
    timeout -k 10 120 tools/batcher_bench 16384 1500 20 5 0 || { cp $O/orig.so brb_framework_amd/libbrb_crypto_gpu.so; exit 1; }
  done
done
cp $O/orig.so brb_framework_amd/libbrb_crypto_gpu.so
