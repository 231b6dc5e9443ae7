#!/bin/bash
# A/B of library builds kept under gpurun_tmp_libs/: per-kernel times of the rc4md5 and rc4 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-ab}; mkdir -p $O
cp brb_framework_amd/libbrb_crypto_gpu.so $O/orig.so
for v in gpurun_tmp_libs/*.so; do
  n=$(basename $v .so)
  cp $v brb_framework_amd/libbrb_crypto_gpu.so
  for op in rc4md5 rc4; do
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n-$op -o run -- python3 bench.py --op $op --no-cpu-baseline > $O/$n-$op.json 2> $O/$n-$op.err || { tail -3 $O/$n-$op.err; exit 1; }
    python3 -c "
import csv
for r in csv.DictReader(open('$O/$n-$op/run_kernel_stats.csv')):
    if 'rc4' in r['Name']: print('$n', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1))"
  done
done
cp $O/orig.so brb_framework_amd/libbrb_crypto_gpu.so
