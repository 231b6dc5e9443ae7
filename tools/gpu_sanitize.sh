#!/bin/bash
# The host runtime under ASan + UBSan WITH a GPU (beyond the CPU leg): the
# sanitized library (make -C brb_framework_amd sanitize: host code instrumented behind -Xarch_host,
# device code untouched) drives the threaded paths that need a device -- the transform batcher
# (arenas, chunk reservation from several threads, zero-copy ranges, pipelined rounds, the
# all-devices router), the host-mode chunk pipelines and their worker threads, the all-devices
# splits -- and any ASan report or UBSan runtime error fails the run.  clang's runtime is put in
# front of whatever the environment already preloads (kept, not replaced).
#   tools/gpu_sanitize.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-san}
mkdir -p "$O"
ASAN_RT="$(cat brb_framework_amd/build-san/asan_runtime.txt)"
[ -f "$ASAN_RT" ] || { echo "no ASan runtime $ASAN_RT"; exit 1; }
export BRB_CRYPTO_LIB="$PWD/brb_framework_amd/build-san/libbrb_crypto_gpu.so"
export ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0:exitcode=86:detect_odr_violation=0:alloc_dealloc_mismatch=0:verify_asan_link_order=0:protect_shadow_gap=0"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=86"
# first: does the runtime start at all in this environment (a plain interpreter, then torch + the library)?
export ASAN_OPTIONS="$ASAN_OPTIONS:log_path=$PWD/$O/asan"
LD_PRELOAD="$ASAN_RT${LD_PRELOAD:+:$LD_PRELOAD}" timeout -k 10 120 python -c "print('asan python ok')" > "$O/probe.log" 2>&1
echo "probe rc=$?"; cat "$O/probe.log"
LD_PRELOAD="$ASAN_RT${LD_PRELOAD:+:$LD_PRELOAD}" timeout -k 10 300 python -c "import torch, brb_framework_amd as b; print('lib', b.crypto.LIB_PATH, b.gpu_available())" > "$O/probe2.log" 2>&1
echo "probe2 rc=$?"; cat "$O/probe2.log"
ls "$O"
LD_PRELOAD="$ASAN_RT${LD_PRELOAD:+:$LD_PRELOAD}" timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 \
    --timeout-method thread tests/test_batcher.py tests/test_host_pipe.py tests/test_all_devices.py \
    tests/test_membuf.py > "$O/pytest_asan.log" 2>&1
rc=$?
tail -3 "$O/pytest_asan.log"
if grep -q -E "ERROR: AddressSanitizer|runtime error:" "$O/pytest_asan.log"; then
    echo "sanitizer report in $O/pytest_asan.log"; exit 1
fi
exit $rc
