#!/bin/bash
# A/B of library builds under gpurun_tmp_libs/*.so by rocprofv3 kernel stats: per build, one bench.py
# run under --kernel-trace --stats; prints the mean duration of every kernel matching <pattern>.
#   tools/gpu_ab_prof.sh <tag> <pattern> <bench.py args...>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-abp}; PAT=$2; shift 2
mkdir -p $O
cp brb_framework_amd/libbrb_crypto_gpu.so $O/intree.so
rc=0
for v in gpurun_tmp_libs/*.so; do
  n=$(basename $v .so)
  cp $v brb_framework_amd/libbrb_crypto_gpu.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- python3 bench.py "$@" --no-cpu-baseline --no-pcie --no-cfg5 > $O/$n.json 2> $O/$n.err || { echo "$n: bench failed (stats still printed)"; tail -2 $O/$n.err; rc=1; }
  [ -f $O/$n/run_kernel_stats.csv ] && python3 -c "
import csv
for r in csv.DictReader(open('$O/$n/run_kernel_stats.csv')):
    if '$PAT' in r['Name']: print('$n', r['Name'][:48], r['Calls'], round(float(r['AverageNs'])/1e3,2))"
done
cp $O/intree.so brb_framework_amd/libbrb_crypto_gpu.so
exit $rc
