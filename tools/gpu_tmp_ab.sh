#!/bin/bash
# round-3 scratch A/B: var-length bucketing (incl. first-round sort) and base64 encode pieces
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_tmp_varbi.sh || exit 1
mkdir -p gpurun_out/r03b64
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_base64.py -m gpu > gpurun_out/r03b64/t.log 2>&1 || { tail -5 gpurun_out/r03b64/t.log; exit 1; }
tail -1 gpurun_out/r03b64/t.log
for v in 2 1 2 1; do
  timeout -k 10 200 python3 bench.py --op base64 --no-cpu-baseline --test-option b64_pieces=$v > gpurun_out/r03b64/b$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r03b64/b$v.json')); print('b64 pieces=$v', d['roofline']['step_us_avg'])"
done
