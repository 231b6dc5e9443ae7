#!/bin/bash
# SURVEY §5 sanitizer leg, CPU only: every line of host code in the
# library -- the compat C and the host side of the HIP runtime (batch_api.hip, host_pipe.hip,
# transform_batcher.hip; device code uninstrumented) -- and the oracle, built with ASan + UBSan on
# clang's runtime (make -C brb_framework_amd sanitize; make -C oracle sanitize), then
#   * the CPU tests that drive them: test_compat, test_abi (with the runtime's and the batcher's
#     argument and refusal paths), test_oracle, test_membuf, test_multigpu (the gloo world-size-2
#     compat leg), test_ref_tables -- with clang's ASan runtime (it carries the UBSan handlers)
#     preloaded into python and the sanitized libraries selected by BRB_CRYPTO_LIB / BRB_ORACLE_LIB;
#   * tests/c/compat_caller.c, itself built with -fsanitize, linked against the sanitized library.
# Any ASan report or UBSan "runtime error" fails the run (halt_on_error; -fno-sanitize-recover).
# Leak checking is off: the python interpreter and torch keep their allocations at exit.
# Usage: tools/sanitize_check.sh [extra pytest args]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
make -s -j8 -C brb_framework_amd all sanitize
make -s -C oracle all sanitize
ASAN_RT="$(cat brb_framework_amd/build-san/asan_runtime.txt)"
[ -f "$ASAN_RT" ] || { echo "[sanitize] FAILED: no clang ASan runtime ($ASAN_RT)"; exit 1; }
[ "$(nm -D brb_framework_amd/build-san/libbrb_crypto_gpu.so | grep -c "__asan_report_load")" -gt 0 ] || { echo "[sanitize] FAILED: library not instrumented"; exit 1; }
for o in brb_md5 batch_api host_pipe transform_batcher; do   # the host runtime's objects are instrumented too
  [ "$(nm "brb_framework_amd/build-san/$o.o" | grep -c "U __asan_report_load")" -gt 0 ] || { echo "[sanitize] FAILED: $o.o not instrumented"; exit 1; }
done
echo "[sanitize] instrumented host objects: compat C + batch_api, host_pipe, transform_batcher (device code untouched)"
export BRB_CRYPTO_LIB="$ROOT/brb_framework_amd/build-san/libbrb_crypto_gpu.so"
export BRB_ORACLE_LIB="$ROOT/oracle/_san/liboracle.so"
export ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0:exitcode=86:detect_odr_violation=0:alloc_dealloc_mismatch=0:verify_asan_link_order=0"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=86"   # one runtime: one exit code
LOG="$(mktemp /tmp/brb_sanitize.XXXXXX)"
echo "[sanitize] pytest under ASan+UBSan (log $LOG)"
LD_PRELOAD="$ASAN_RT" python -m pytest -q -p no:cacheprovider -m "not gpu" \
    tests/test_compat.py tests/test_abi.py tests/test_oracle.py tests/test_membuf.py tests/test_multigpu.py \
    tests/test_ref_tables.py "$@" 2>&1 | tee "$LOG" | tail -3
if grep -q -E "ERROR: AddressSanitizer|runtime error:" "$LOG"; then
    echo "[sanitize] FAILED: sanitizer report in $LOG"; exit 1
fi
echo "[sanitize] positive control: a 200-byte BRB_MD5Update over a 100-byte heap buffer must be caught"
set +e
LD_PRELOAD="$ASAN_RT" python - > "$LOG.ctl" 2>&1 <<'PY'
import ctypes, os
L = ctypes.CDLL(os.environ["BRB_CRYPTO_LIB"])
libc = ctypes.CDLL(None)
libc.malloc.restype = ctypes.c_void_p
p = libc.malloc(100)
ctx = ctypes.create_string_buffer(168)
L.BRB_MD5Init(ctx)
L.BRB_MD5Update(ctx, ctypes.c_void_p(p), ctypes.c_ulong(200))
PY
rc=$?
set -e
if [ "$rc" != 86 ] || ! grep -q "heap-buffer-overflow" "$LOG.ctl"; then
    echo "[sanitize] FAILED: the instrumented library did not report the overflow (exit $rc)"; tail -20 "$LOG.ctl"; exit 1
fi
echo "[sanitize] positive control reported: $(grep -m1 -o 'heap-buffer-overflow.*' "$LOG.ctl" | cut -c1-60) ... $(grep -m1 -o 'in BRB_MD5[A-Za-z]*' "$LOG.ctl")"
echo "[sanitize] C caller built with -fsanitize=address,undefined"
EXE="$(mktemp /tmp/brb_caller_san.XXXXXX)"
/opt/rocm/llvm/bin/clang -std=c99 -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined \
    -shared-libsan -Wall -Werror -I include tests/c/compat_caller.c -L "$(dirname "$BRB_CRYPTO_LIB")" -lbrb_crypto_gpu \
    -Wl,-rpath,"$(dirname "$BRB_CRYPTO_LIB")" -Wl,-rpath,"$(dirname "$ASAN_RT")" -o "$EXE"
"$EXE" > "$LOG.caller" 2>&1 || { echo "[sanitize] FAILED: C caller exit $?"; tail -30 "$LOG.caller"; exit 1; }
if grep -q -E "ERROR: AddressSanitizer|runtime error:" "$LOG.caller"; then
    echo "[sanitize] FAILED: sanitizer report in $LOG.caller"; exit 1
fi
echo "[sanitize] C caller: $(wc -l < "$LOG.caller") result lines, no sanitizer report"
rm -f "$EXE" "$LOG" "$LOG.caller" "$LOG.ctl"
echo "[sanitize] OK"
