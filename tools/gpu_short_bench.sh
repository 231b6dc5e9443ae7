#!/bin/bash
# The headline at the driver's flags (--steps 20 --warmup 5) against longer warm-ups, with and without
# the cfg5 leg before it: where the short run's slower launches come from.
#   tools/gpu_short_bench.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-short}
mkdir -p "$OUT"
run() {   # name, args...
    local n=$1; shift
    timeout -k 10 240 python bench.py --no-pcie --no-cpu-baseline "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" || return 1
    python3 - "$OUT/$n.json" "$n" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
c = d.get("cfg5", {})
print(f"{sys.argv[2]:14s} value {d['value']:8.1f} ms/step {d['ms_per_step']*1e3:6.2f} us  ev {r['launch_us_avg']:6.2f} us  all_k {r['launch_us_avg_all_k']:6.2f} us  cfg5 {c.get('launch_us_avg', '-')}")
PY
}
for i in 1 2; do
    run "d20w5_$i" --steps 20 --warmup 5 &&
    run "n20w5_$i" --steps 20 --warmup 5 --no-cfg5 &&
    run "n20w20k_$i" --steps 20 --warmup 20000 --no-cfg5 &&
    run "d20w20k_$i" --steps 20 --warmup 20000 &&
    run "d2000w5_$i" --steps 2000 --warmup 5 || exit 1
done
