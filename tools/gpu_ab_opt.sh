#!/bin/bash
# Interleaved A/B of one library build under values of a test option (BRB_CryptoGPU_TestOption,
# passed as bench.py --test-option NAME=VALUE):
#   tools/gpu_ab_opt.sh <tag> <rounds> <option> "<value> <value> ..." <bench.py args...>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-abo}; R=${2:-3}; V=$3; VALS=$4; shift 4
mkdir -p $O
for r in $(seq 1 $R); do
  for x in $VALS; do
    timeout -k 10 200 python3 bench.py "$@" --test-option $V=$x --no-cpu-baseline --no-pcie --no-cfg5 > $O/$V-$x-$r.json 2> $O/$V-$x-$r.err || { tail -3 $O/$V-$x-$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$V-$x-$r.json')); print('$V=$x', $r, d['value'], d['unit'], d['roofline'].get('launch_us_avg', d['roofline'].get('step_us_avg')))"
  done
done
