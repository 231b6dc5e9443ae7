#!/bin/bash
# round-3 scratch A/B: fixed-stride line kernel, tickets per workgroup (0) vs device-wide (1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03tk
for v in 0 1 0 1 0 1; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-pcie --test-option line_tickets=$v > gpurun_out/r03tk/t$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r03tk/t$v.json')); print('tickets $v cfg2', d['roofline']['launch_us_avg'], 'cfg5', d['cfg5']['launch_us_avg'], d['cfg5']['roofline_frac'])"
done
