#!/bin/bash
# Round 4, first kernel pass: parity of the new kernels (line-staged segments / MetaData, the lean
# 64-byte digest), then interleaved A/B of each against the kernel it replaces, then valu_mix.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04a}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_segments.py tests/test_metadata.py "tests/test_gpu_parity.py" -x -q \
    --timeout 300 --timeout-method thread -k "segments or unpack or cfg3 or short or small or 64 or edge" > $O/pytest.log 2>&1 \
    || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_ab_opt.sh ${1:-r04a}/seg 2 seg_line "1 0" --op md5seg || exit 1
bash tools/gpu_ab_opt.sh ${1:-r04a}/md 2 seg_line "1 0" --op metadata || exit 1
bash tools/gpu_ab_opt.sh ${1:-r04a}/b64 3 b64_kernel "1 0" --config 3 || exit 1
timeout -k 10 120 tools/mb/valu_mix > $O/valu_mix.txt 2>&1 || { echo "valu_mix failed"; exit 1; }
grep -E "4 add|5 add|7 add|split|MD5 mix|3 add" $O/valu_mix.txt
echo done
