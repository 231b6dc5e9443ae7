#!/bin/bash
# Every bench line of DESIGN.md §5 on one box: cfg2 (default, with cfg5 and host-inclusive rates),
# SHA-1, cfg3, cfg4, f1 RC4 / RC4+MD5, f4 MetaData / base64, cfg1.  Each step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-benchall}
mkdir -p "$OUT"
timeout -k 10 300 python bench.py > "$OUT/cfg2.json" 2> "$OUT/cfg2.err" && echo "cfg2 ok" &&
timeout -k 10 300 python bench.py --op sha1 --no-cfg5 > "$OUT/sha1.json" 2> "$OUT/sha1.err" && echo "sha1 ok" &&
timeout -k 10 300 python bench.py --config 3 > "$OUT/cfg3.json" 2> "$OUT/cfg3.err" && echo "cfg3 ok" &&
timeout -k 10 300 python bench.py --config 4 > "$OUT/cfg4.json" 2> "$OUT/cfg4.err" && echo "cfg4 ok" &&
timeout -k 10 300 python bench.py --op rc4 > "$OUT/rc4.json" 2> "$OUT/rc4.err" && echo "rc4 ok" &&
timeout -k 10 300 python bench.py --op rc4md5 > "$OUT/rc4md5.json" 2> "$OUT/rc4md5.err" && echo "rc4md5 ok" &&
timeout -k 10 300 python bench.py --op metadata > "$OUT/metadata.json" 2> "$OUT/metadata.err" && echo "metadata ok" &&
timeout -k 10 300 python bench.py --op md5seg > "$OUT/md5seg.json" 2> "$OUT/md5seg.err" && echo "md5seg ok" &&
timeout -k 10 300 python bench.py --op base64 > "$OUT/base64.json" 2> "$OUT/base64.err" && echo "base64 ok" &&
timeout -k 10 300 python bench.py --op md5var --no-cfg5 > "$OUT/md5var.json" 2> "$OUT/md5var.err" && echo "md5var ok" &&
timeout -k 10 300 python bench.py --op sha1var --no-cfg5 > "$OUT/sha1var.json" 2> "$OUT/sha1var.err" && echo "sha1var ok" &&
timeout -k 10 300 python bench.py --config 1 > "$OUT/cfg1.json" 2> "$OUT/cfg1.err" && echo "cfg1 ok"
