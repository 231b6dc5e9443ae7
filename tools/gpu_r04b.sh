#!/bin/bash
# Round 4: parity of the line-staged segment / MetaData kernels, A/B vs the per-lane kernels, PMC.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r04b}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_segments.py tests/test_metadata.py -x -q \
    --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_ab_opt.sh $T/seg 2 seg_line "1 0" --op md5seg || exit 1
bash tools/gpu_ab_opt.sh $T/md 2 seg_line "1 0" --op metadata || exit 1
bash tools/gpu_pmc.sh $T/pmc_seg --op md5seg > /dev/null || exit 1
bash tools/gpu_pmc.sh $T/pmc_md --op metadata > /dev/null || exit 1
echo done
