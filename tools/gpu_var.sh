#!/bin/bash
# Kernel durations of the fixed-stride and variable-length digest paths (tools/var_bench.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-var}; mkdir -p $O
shift
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 tools/var_bench.py "$@" > $O/out.txt 2>&1 || { tail -5 $O/out.txt; exit 1; }
cat $O/out.txt | tail -4
python3 -c "
import csv
for r in csv.DictReader(open('$O/p/run_kernel_stats.csv')):
    print(r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1e3,2))"
