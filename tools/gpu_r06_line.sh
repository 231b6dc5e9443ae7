#!/bin/bash
# Round 6: the line kernel with its group-invariant setup hoisted -- parity of
# every fixed-stride line shape, then the in-process interleaved A/B against round 5's form
# (tools/mb/line_ab) on the cfg5 shard and cfg2, then bench.py's cfg2 and cfg5-shard lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06line}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_all_devices.py \
    -k "line_kernel or cfg5_full or cfg2_full or large_batch or many_groups or edge_lengths or unaligned or line_forced or golden_edge" \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 tools/mb/line_ab 1048576 1500 ${ROUNDS:-5} 40 > $O/line_ab_cfg5.txt 2>&1 || { tail -5 $O/line_ab_cfg5.txt; exit 1; }
grep -E "^n=|MEDIAN" $O/line_ab_cfg5.txt
timeout -k 10 200 tools/mb/line_ab 65536 1500 ${ROUNDS:-5} 400 > $O/line_ab_cfg2.txt 2>&1 || { tail -5 $O/line_ab_cfg2.txt; exit 1; }
grep -E "^n=|MEDIAN" $O/line_ab_cfg2.txt
timeout -k 10 200 python3 bench.py --records-per-gpu 1048576 --no-cpu-baseline --no-pcie --no-cfg5 > $O/cfg5.json 2> $O/cfg5.err || { tail -3 $O/cfg5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/cfg5.json')); r=d['roofline']; print('bench cfg5 shard', round(r['launch_us_avg'],2), r['frac'])"
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-pcie > $O/cfg2.json 2> $O/cfg2.err || { tail -3 $O/cfg2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/cfg2.json')); r=d['roofline']; print('bench cfg2', round(r['launch_us_avg'],2), r['frac'], 'cfg5', d.get('cfg5'))"
