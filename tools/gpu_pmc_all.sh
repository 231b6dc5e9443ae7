#!/bin/bash
# Every PMC pass bench.py's roofline.traffic / roofline.compute read (tools/gpu_pmc.sh: one rocprofv3
# --pmc pass per counter group, kernel trace only).
#   tools/gpu_pmc_all.sh <tag> [pass ...]   -> gpurun_out/<tag>/<pass>/  (default: every pass)
# then, here: python3 tools/collect_profiles.py gpurun_out/<tag> <round tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-pmcall}; shift
declare -A ARGS=(
  [pmc2]="--config 2"        [pmc2s]="--config 2 --op sha1"  [pmc3]="--config 3"
  [pmc4]="--config 4"        [pmc_rc4]="--op rc4"            [pmc_rc4md5]="--op rc4md5"
  [pmc_md]="--op metadata"   [pmc_seg]="--op md5seg"         [pmc_b64]="--op base64"
  [pmc_md5var]="--op md5var" [pmc_sha1var]="--op sha1var"
  [pmc5]="--records-per-gpu 1048576"
)
PASSES=${@:-pmc2 pmc2s pmc3 pmc4 pmc_rc4 pmc_rc4md5 pmc_md pmc_seg pmc_b64 pmc_md5var pmc_sha1var pmc5}
for d in $PASSES; do
  bash tools/gpu_pmc.sh "$T/$d" ${ARGS[$d]} > /dev/null || { echo "$d failed"; exit 1; }
  echo "$d ok"
done
