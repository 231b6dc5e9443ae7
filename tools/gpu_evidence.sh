#!/bin/bash
# Every kept bench line under rocprofv3 --kernel-trace --stats, each with its timed region marked
# (bench.py --mark-timed-region), then tools/collect_evidence.py recomputes each line's fraction
# from the rocprof mean of exactly its timed dispatches.  Each step has its own time limit; a failed
# step ends the script.
#   tools/gpu_evidence.sh <tag> [line ...]     (default: every line)
#   PLAIN=gpurun_out/<tag2> ...: also join the unprofiled lines of tools/gpu_bench_all.sh <tag2>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-ev}; shift
O=gpurun_out/$TAG
mkdir -p "$O"
declare -A ARGS=(
  [cfg2]=""                      [sha1]="--op sha1 --no-cfg5"    [cfg3]="--config 3"
  [cfg4]="--config 4"            [rc4]="--op rc4"                [rc4md5]="--op rc4md5"
  [metadata]="--op metadata"     [md5seg]="--op md5seg"          [base64]="--op base64"
  [md5var]="--op md5var"         [sha1var]="--op sha1var"
)
LINES=${@:-cfg2 sha1 cfg3 cfg4 rc4 rc4md5 metadata md5seg base64 md5var sha1var}
for l in $LINES; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$l" -o run -- \
      python3 bench.py ${ARGS[$l]} --mark-timed-region > "$O/$l.json" 2> "$O/$l.err" \
      || { echo "$l failed"; tail -5 "$O/$l.err"; exit 1; }
  echo "$l ok"
done
timeout -k 10 300 python3 bench.py --config 1 > "$O/cfg1.json" 2> "$O/cfg1.err" && echo "cfg1 ok"
timeout -k 10 300 python3 tools/collect_evidence.py "$O" "$O/evidence" $PLAIN || exit 1
# the raw traces (tens of MB per line) stay on the box; the per-region summaries come back
find "$O" -name run_kernel_trace.csv -delete
