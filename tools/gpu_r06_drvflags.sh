#!/bin/bash
# Round 6: the headline at the driver flags (--steps 20 --warmup 5), with and without the cfg5 leg
# before it, interleaved three times (the 20-step region varied 20.1-24.1 us per launch).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06drv2
for i in 1 2 3; do
  for v in cfg5 nocfg5; do
    extra=""; [ $v = nocfg5 ] && extra="--no-cfg5"
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 $extra > gpurun_out/r06drv2/$v-$i.json 2> gpurun_out/r06drv2/$v-$i.err || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/r06drv2/$v-$i.json')); print('$v', $i, d['value'], d['roofline']['launch_us_avg'], d['roofline']['frac'])
"
  done
done
