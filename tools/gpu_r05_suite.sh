#!/bin/bash
# Round-5 closing pass on the committed tree: every GPU test, smoke, the default bench line and a
# two-rank rehearsal of the bench on the one GPU.  Each step has its own time limit; a failed step
# ends the script.
#   tools/gpu_r05_suite.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05suite}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 && echo "pytest ok" &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && echo "bench ok" && cat "$OUT/bench.json" &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-pcie > "$OUT/bench_n2.json" 2> "$OUT/bench_n2.err" && echo "bench n2 ok" && cat "$OUT/bench_n2.json"
rc=$?
tail -3 "$OUT/pytest_gpu.log"
exit $rc
