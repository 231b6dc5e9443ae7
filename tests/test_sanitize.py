"""SURVEY §5 sanitizer leg on the CPU build: tools/sanitize_check.sh builds the
host compat C and the oracle with ASan + UBSan, runs the compat / ABI / oracle / MemBuffer /
multi-process tests and the unchanged C caller against those builds, and checks that a planted
heap overflow is reported (so a clean run means the instrumentation was live).  The reference quirks
those tests drive are md5.c:114-121 (UpdateLowerText's 128-byte buffer), sha1.c:157-158 (in-place
blocks) and mem_buf.c:1518-1542 (the +2 words past the data)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_code_clean_under_asan_ubsan():
    env = {k: v for k, v in os.environ.items() if k not in ("BRB_CRYPTO_LIB", "BRB_ORACLE_LIB", "LD_PRELOAD")}
    out = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize_check.sh")], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=900)
    tail = (out.stdout + out.stderr)[-3000:]
    assert out.returncode == 0, tail
    assert "[sanitize] OK" in out.stdout, tail
    assert "positive control reported: heap-buffer-overflow" in out.stdout, tail
