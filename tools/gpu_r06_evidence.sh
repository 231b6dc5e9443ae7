#!/bin/bash
# Round-6 evidence on one box, in parts (each fits one gpurun call; every step has its own limit):
#   tools/gpu_r06_evidence.sh <tag> pmc    every PMC pass (tools/gpu_pmc_all.sh, now with the cfg5 shard)
#   tools/gpu_r06_evidence.sh <tag> lines  every bench line unprofiled, then under rocprofv3 with its
#                                          timed region marked (tools/gpu_evidence.sh)
#   tools/gpu_r06_evidence.sh <tag> suite  the whole -m gpu suite, smoke(), the default bench line and a
#                                          two-rank rehearsal (tools/gpu_r05_suite.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r06ev}
case "${2:-pmc}" in
  pmc)   bash tools/gpu_pmc_all.sh "$T/pmc" && echo "pmc ok" &&
         timeout -k 10 120 python3 tools/collect_profiles.py "gpurun_out/$T/pmc" r06 > "gpurun_out/$T/pmc_traffic.json" && echo "collected" ;;
  lines) bash tools/gpu_bench_all.sh "$T/plain" && echo "plain ok" &&
         PLAIN=gpurun_out/$T/plain bash tools/gpu_evidence.sh "$T/ev" && echo "evidence ok" ;;
  suite) bash tools/gpu_r05_suite.sh "$T/suite" ;;
  *)     echo "unknown part $2"; exit 2 ;;
esac
