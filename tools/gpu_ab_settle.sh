#!/bin/bash
# Interleaved A/B of the settle before an explicit W: bench_prev.py (a copy of the previous bench.py, made
# by hand: git show <rev>:bench.py > bench_prev.py) against bench.py, three rounds at the driver's flags.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/absettle
for r in 1 2 3; do
  for v in prev new; do
    b=bench.py; [ $v = prev ] && b=bench_prev.py
    timeout -k 10 200 python $b --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-pcie > gpurun_out/absettle/$v-$r.json 2> gpurun_out/absettle/$v-$r.err || exit 1
    python3 -c "
import json;d=json.loads(open('gpurun_out/absettle/$v-$r.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$v-$r',d['value'],d['ms_per_step'],r['launch_us_avg'],r['frac'],d['settle']['launches'])"
  done
done
