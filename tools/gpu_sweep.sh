#!/bin/bash
# Measurement sweep for DESIGN.md's table: every bench workload once, JSON per run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-sweep}
mkdir -p "$OUT"
run() {   # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" && echo "$name ok: $(head -c 160 "$OUT/$name.json")"
}
run cfg2_md5 --no-pcie --no-cpu-baseline &&
run cfg2_md5_2s --two-stream --no-pcie --no-cpu-baseline &&
run cfg2_sha1 --op sha1 --no-pcie --no-cpu-baseline &&
run cfg3_md5 --config 3 --no-pcie --no-cpu-baseline &&
run cfg5_md5 --config 5 --no-pcie --no-cpu-baseline &&
run cfg4_bf --config 4 &&
run f1_rc4 --op rc4 --no-cpu-baseline &&
run f1_rc4md5 --op rc4md5 &&
run f2_batcher --op batcher
