#!/bin/bash
# the zero-copy pipelined batcher round (tools/batcher_bench, 16 384 connections
# x one 1530-byte frame in + one 1500-byte payload out per round, 1 submit thread) under
# rocprofv3 --kernel-trace --memory-copy-trace: where a round's time goes (tools/batcher_timeline.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-bt}; mkdir -p $O
for m in "1 1 1" "0 1 4"; do
  set -- $m
  timeout -k 10 120 tools/batcher_bench 16384 1500 20 5 $1 $2 $3 > $O/plain_zc$1_p$2_t$3.json 2>&1 || { tail -5 $O/plain_zc$1_p$2_t$3.json; exit 1; }
  tail -1 $O/plain_zc$1_p$2_t$3.json
  timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr_zc$1_p$2_t$3 -o run -- \
      tools/batcher_bench 16384 1500 20 5 $1 $2 $3 > $O/tr_zc$1_p$2_t$3.json 2>&1 || { tail -5 $O/tr_zc$1_p$2_t$3.json; exit 1; }
  tail -1 $O/tr_zc$1_p$2_t$3.json
done
echo done
