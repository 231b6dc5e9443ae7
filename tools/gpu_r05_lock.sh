#!/bin/bash
# Round 5: the line kernel's static split with SIMD partners in lockstep (test option line_lock) --
# parity, then an interleaved A/B on the cfg5 shard and cfg2, then the per-wave end probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05lock}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
    -k "line_lock or cfg5_full" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2 3; do
  for x in ${LOCKS:-0 1 2 4}; do
    timeout -k 10 200 python3 bench.py --records-per-gpu 1048576 --test-option line_lock=$x --no-cpu-baseline --no-pcie --no-cfg5 \
        > $O/cfg5-$x-$r.json 2> $O/cfg5-$x-$r.err || { tail -3 $O/cfg5-$x-$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/cfg5-$x-$r.json')); r=d['roofline']; print('cfg5 line_lock=$x', $r, round(r['launch_us_avg'],2), r['frac'])"
  done
done
[ -n "$PROBE" ] && { timeout -k 10 300 tools/mb/lprobe5 1048576 1500 pool > $O/lprobe.txt 2>&1; grep -E "^LINE|per-WG" $O/lprobe.txt; }
true
