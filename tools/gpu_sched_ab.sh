#!/bin/bash
# A/B of library builds that differ only in hipcc's AMDGPU machine-scheduler strategy
# (-mllvm --amdgpu-sched-strategy=..., builds under gpurun_tmp_libs/): digest/Blowfish parity per
# build, then interleaved bench rounds for cfg2 MD5, SHA-1, cfg3, cfg4 and the RC4 pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_ab_parity.sh sched_t tests/test_gpu_parity.py -k "edge or cfg2 or blowfish_batch" &&
bash tools/gpu_ab_libs.sh sched_a 3 &&
bash tools/gpu_ab_libs.sh sched_s 2 --op sha1 &&
bash tools/gpu_ab_libs.sh sched_c3 2 --config 3 &&
bash tools/gpu_ab_libs.sh sched_c4 1 --config 4 &&
bash tools/gpu_ab_libs.sh sched_rc4 1 --op rc4
