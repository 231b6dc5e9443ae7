#!/bin/bash
# Quick GPU pass: parity tests + cfg2/cfg3/cfg5-shard benches (no CPU baseline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-quick}
mkdir -p "$OUT"
timeout -k 10 900 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
for c in "--config 2" "--config 2 --op sha1" "--config 3" "--config 5" ; do
  timeout -k 10 300 python bench.py $c --no-cpu-baseline --no-pcie --two-stream --steps 100 > "$OUT/b.json" 2> "$OUT/b.err" || { cat "$OUT/b.err"; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/b.json')); r=d['roofline']; print('$c', d['value'], d['unit'], d.get('mrecords_per_s'), 'kern_us', r.get('launch_us_avg', r.get('step_us_avg')), 'frac', r['frac'], 'ms_step', d['ms_per_step'], '2str', d.get('two_stream_throughput', {}).get('value'))"
done
