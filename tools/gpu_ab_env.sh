#!/bin/bash
# Interleaved A/B of one library build under two values of an environment switch:
#   tools/gpu_ab_env.sh <tag> <rounds> <VAR> <value A> <value B> <bench.py args...>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-abe}; R=${2:-3}; V=$3; A=$4; B=$5; shift 5
mkdir -p $O
for r in $(seq 1 $R); do
  for x in $A $B; do
    env $V=$x timeout -k 10 200 python3 bench.py "$@" --no-cpu-baseline --no-pcie --no-cfg5 > $O/$V-$x-$r.json 2> $O/$V-$x-$r.err || { tail -3 $O/$V-$x-$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$V-$x-$r.json')); print('$V=$x', $r, d['value'], d['unit'], d['roofline'].get('launch_us_avg', d['roofline'].get('step_us_avg')))"
  done
done
