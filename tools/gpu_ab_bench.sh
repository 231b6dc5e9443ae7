#!/bin/bash
# Interleaved A/B of library builds kept under gpurun_tmp_libs/ on one bench command:
#   tools/gpu_ab_bench.sh <tag> <rounds> <bench.py args...>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-abb}; R=${2:-3}; shift 2
mkdir -p $O
cp brb_framework_amd/libbrb_crypto_gpu.so $O/orig.so
for r in $(seq 1 $R); do
  for v in gpurun_tmp_libs/*.so; do
    n=$(basename $v .so)
    cp $v brb_framework_amd/libbrb_crypto_gpu.so
    timeout -k 10 200 python3 bench.py "$@" --no-cpu-baseline --no-pcie > $O/$n-$r.json 2> $O/$n-$r.err || { tail -3 $O/$n-$r.err; cp $O/orig.so brb_framework_amd/libbrb_crypto_gpu.so; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$n-$r.json')); print('$n', $r, d['value'], d['unit'], d['roofline'].get('launch_us_avg', d['roofline'].get('step_us_avg')))"
  done
done
cp $O/orig.so brb_framework_amd/libbrb_crypto_gpu.so
