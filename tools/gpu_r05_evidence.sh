#!/bin/bash
# Round-5 evidence pass on one box: every PMC pass (kernel identities recorded; collected into this
# box's profiles/pmc_traffic.json, which the lines then read -- rerun collect_profiles.py here on the
# merged gpurun_out/<tag>/pmc to get the same file), then every bench line
# unprofiled, then every line under rocprofv3 with its timed region marked.  Each step has its own
# time limit inside the called scripts; a failed step ends the script.
#   tools/gpu_r05_evidence.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05ev}
bash tools/gpu_pmc_all.sh "$T/pmc" && echo "pmc ok" &&
timeout -k 10 120 python3 tools/collect_profiles.py "gpurun_out/$T/pmc" r05 > "gpurun_out/$T/pmc_traffic.json" && echo "collected" &&
bash tools/gpu_bench_all.sh "$T/plain" && echo "plain ok" &&
PLAIN=gpurun_out/$T/plain bash tools/gpu_evidence.sh "$T/ev" && echo "evidence ok"
