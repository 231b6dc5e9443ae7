#!/bin/bash
# Every bench line at the driver's flags (--steps 20 --warmup 5, so each runs its settle first):
# the lines' own checks (digests, round trips, validation) must still pass after the settle's
# launches.  Each step has its own time limit; a failed step ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-settle_ops}
mkdir -p "$OUT"
for a in "--config 2" "--op sha1 --no-cfg5" "--config 3" "--config 4" "--op rc4" "--op rc4md5" "--op metadata" \
         "--op md5seg" "--op base64" "--op md5var" "--op sha1var"; do
    n=$(echo "$a" | tr -d ' -')
    timeout -k 10 300 python bench.py $a --steps 20 --warmup 5 --no-cpu-baseline --no-pcie > "$OUT/$n.json" 2> "$OUT/$n.err" \
        || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
    python3 -c "
import json,sys;d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]);r=d.get('roofline') or {}
print('$n', d['value'], d['unit'], 'ms/step', d['ms_per_step'], 'frac', r.get('frac'), 'settle', (d.get('settle') or {}).get('launches'))"
done
