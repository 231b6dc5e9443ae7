#!/bin/bash
# Interleaved A/B of two bench.py versions at the driver's flags (--steps 20 --warmup 5): the previous one
# copied to bench_prev_order.py at the repo root (not kept), and the current one.
set -o pipefail
mkdir -p gpurun_out/ord
for r in 1 2 3 4; do
  for v in old new; do
    if [ $v = old ]; then B=bench_prev_order.py; else B=bench.py; fi
    timeout -k 10 200 python $B --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-pcie > gpurun_out/ord/$v-$r.json 2> gpurun_out/ord/$v-$r.err || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['launch_us_avg'], d['cfg5']['launch_us_avg'])" gpurun_out/ord/$v-$r.json $v
  done
done
