#!/bin/bash
# Interleaved A/B of library builds kept under gpurun_tmp_libs/*.so (git-ignored, they travel with
# the snapshot): R rounds, each runs bench.py once per build with the given bench arguments and
# prints the per-launch time.  The in-tree library is restored at the end.
#   tools/gpu_ab_libs.sh <tag> <rounds> <bench.py args...>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-abl}; R=${2:-3}; shift 2
mkdir -p $O
cp brb_framework_amd/libbrb_crypto_gpu.so $O/intree.so
rc=0
for r in $(seq 1 $R); do
  for v in gpurun_tmp_libs/*.so; do
    n=$(basename $v .so)
    cp $v brb_framework_amd/libbrb_crypto_gpu.so
    timeout -k 10 200 python3 bench.py "$@" --no-cpu-baseline --no-pcie --no-cfg5 > $O/$n-$r.json 2> $O/$n-$r.err || { tail -3 $O/$n-$r.err; rc=1; break 2; }
    python3 -c "import json; d=json.load(open('$O/$n-$r.json')); print('$n', $r, d['value'], d['unit'], d['roofline'].get('launch_us_avg', d['roofline'].get('step_us_avg')))"
  done
done
cp $O/intree.so brb_framework_amd/libbrb_crypto_gpu.so
exit $rc
