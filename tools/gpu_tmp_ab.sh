#!/bin/bash
# round-3 scratch A/B: base64 group kernels -- pieces per pass, nontemporal stores, lanes per record
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03b64d
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_base64.py -m gpu > gpurun_out/r03b64d/t.log 2>&1 || { tail -30 gpurun_out/r03b64d/t.log; exit 1; }
tail -1 gpurun_out/r03b64d/t.log
for cfg in "0 -1" "1 -1" "2 -1" "3 -1" "0 4" "1 4" "1 6" "3 4" "0 -1" "1 -1" "2 -1" "3 -1"; do
  set -- $cfg
  timeout -k 10 200 python3 bench.py --op base64 --no-cpu-baseline --test-option b64_variant=$1 --test-option b64_group=$2 > gpurun_out/r03b64d/v$1g$2.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r03b64d/v$1g$2.json')); print('variant $1 group $2', d['roofline']['step_us_avg'], d['roofline']['frac'])"
done
