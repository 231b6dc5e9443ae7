#!/bin/bash
# Every PMC pass bench.py's roofline.traffic / roofline.compute read (tools/gpu_pmc.sh: one rocprofv3
# --pmc pass per counter group, kernel trace only), then tools/collect_profiles.py on the box.
#   tools/gpu_pmc_all.sh <tag>      -> gpurun_out/<tag>/pmc*/, gpurun_out/<tag>/pmc_traffic.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-pmcall}
for spec in "pmc2:--config 2" "pmc2s:--config 2 --op sha1" "pmc3:--config 3" "pmc4:--config 4" \
            "pmc_rc4:--op rc4" "pmc_rc4md5:--op rc4md5" "pmc_md:--op metadata" "pmc_seg:--op md5seg" \
            "pmc_b64:--op base64" "pmc_md5var:--op md5var" "pmc_sha1var:--op sha1var"; do
  d=${spec%%:*}; a=${spec#*:}
  bash tools/gpu_pmc.sh "$T/$d" $a > /dev/null || { echo "$d failed"; exit 1; }
  echo "$d ok"
done
