#!/bin/bash
# Round 5: the line kernel's tail pool -- parity, then an interleaved A/B of test option line_pool on
# the cfg5 shard (1 Mi x 1500 B per GPU) and cfg2, then the per-wave end probe without / with the pool.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05pool}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
    -k "line_pool or cfg5 or line_kernel_short or many_groups or cfg2_full" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for r in 1 2 3; do
  for x in 0 4 8 16; do
    timeout -k 10 200 python3 bench.py --records-per-gpu 1048576 --test-option line_pool=$x --no-cpu-baseline --no-pcie --no-cfg5 \
        > $O/cfg5-$x-$r.json 2> $O/cfg5-$x-$r.err || { tail -3 $O/cfg5-$x-$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/cfg5-$x-$r.json')); r=d['roofline']; print('cfg5 line_pool=$x', $r, round(r['launch_us_avg'],2), r['frac'])"
  done
done
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-pcie --no-cfg5 > $O/cfg2.json 2> $O/cfg2.err && python3 -c "import json; d=json.load(open('$O/cfg2.json')); r=d['roofline']; print('cfg2', round(r['launch_us_avg'],2), r['frac'])"
timeout -k 10 300 tools/mb/lprobe5 1048576 1500 pool > $O/lprobe_pool.txt 2>&1; grep -E "^LINE|per-WG" $O/lprobe_pool.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log
