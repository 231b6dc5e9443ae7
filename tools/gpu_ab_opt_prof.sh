#!/bin/bash
# A/B of one library build under values of a test option, by rocprofv3 kernel stats: per value, one
# bench.py run under --kernel-trace --stats; prints the mean duration of every kernel matching <pattern>.
#   tools/gpu_ab_opt_prof.sh <tag> <pattern> <option> "<value> <value> ..." <bench.py args...>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-abop}; PAT=$2; OPT=$3; VALS=$4; shift 4
mkdir -p $O
for x in $VALS; do
  n=$OPT-$x
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- python3 bench.py "$@" --test-option $OPT=$x --no-cpu-baseline --no-pcie --no-cfg5 > $O/$n.json 2> $O/$n.err || { echo "$n: bench failed"; tail -2 $O/$n.err; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$O/$n/run_kernel_stats.csv')):
    if '$PAT' in r['Name']: print('$n', r['Name'][:48], r['Calls'], round(float(r['AverageNs'])/1e3,2))"
done
