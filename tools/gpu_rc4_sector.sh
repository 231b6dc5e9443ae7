#!/bin/bash
# A/B of the RC4 pass output sink (SectorSnk vs Snk): HBM (bench.py --op rc4) and the zero-copy RC4
# batcher (outputs written into page-locked host memory over PCIe), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-rc4sector}
mkdir -p "$OUT"
LIB=$PWD/brb_framework_amd
for rep in 1 2; do
  for v in 0 1; do
    BRB_TEST_RC4_SECTOR=$v timeout -k 10 200 python bench.py --op rc4 --no-cpu-baseline > "$OUT/hbm_$v.$rep.json" 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('$OUT/hbm_$v.$rep.json')); print('hbm sector=$v', d['roofline']['step_us_avg'])"
    BRB_TEST_RC4_SECTOR=$v timeout -k 10 200 ./tools/batcher_bench 16384 1500 20 5 1 0 1 1 > "$OUT/zc_$v.$rep.json" || exit 1
    BRB_TEST_RC4_SECTOR=$v timeout -k 10 200 ./tools/batcher_bench 16384 1500 20 5 1 1 1 1 > "$OUT/zcp_$v.$rep.json" || exit 1
    python3 -c "import json; a=json.load(open('$OUT/zc_$v.$rep.json')); b=json.load(open('$OUT/zcp_$v.$rep.json')); print('zc rc4 sector=$v', a['round_ms_mean'], a['payload_gib_s'], 'pipelined', b['round_ms_mean'], b['payload_gib_s'])"
  done
done
