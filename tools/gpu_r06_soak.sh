#!/bin/bash
# Round 6: soaks of the round's changed kernels against the oracle -- the fuzz tests over fresh seeds
# (every batch entry point; default and 8x batch sizes), the batcher's event loop in all eight modes,
# and several host threads calling the library at once.  Each soak has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06soak}
mkdir -p $O
timeout -k 10 330 python -u tools/fuzz_soak.py 240 60000 > $O/fuzz_soak.txt 2>&1 && tail -1 $O/fuzz_soak.txt &&
timeout -k 10 270 python -u tools/fuzz_soak.py --scale=8 180 61000 > $O/fuzz_soak_x8.txt 2>&1 && tail -1 $O/fuzz_soak_x8.txt &&
timeout -k 10 240 python -u tools/fuzz_soak.py 150 62000 batcher > $O/fuzz_soak_batcher.txt 2>&1 && tail -1 $O/fuzz_soak_batcher.txt &&
timeout -k 10 200 python -u tools/thread_soak.py 120 8 > $O/thread_soak.txt 2>&1 && tail -2 $O/thread_soak.txt
