#!/bin/bash
# Round evidence pass: parity tests, smoke, default bench, rocprofv3 kernel stats of the bench,
# PMC passes (FETCH/WRITE sizes + SQ counters) for the bench workload and cfg4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-round}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 && echo "pytest ok" &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && echo "bench ok" && cat "$OUT/bench.json" &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-pcie > "$OUT/bench_n2.json" 2> "$OUT/bench_n2.err" && echo "bench n2 ok" && cat "$OUT/bench_n2.json" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-pcie --no-cfg5 > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" && echo "rocprof ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof4" -o run --output-format csv -- \
    python3 bench.py --config 4 --no-cpu-baseline > "$OUT/bench4_prof.json" 2> "$OUT/bench4_prof.err" && echo "rocprof4 ok" &&
bash tools/gpu_pmc.sh "${1:-round}/pmc2" --config 2 > /dev/null && echo "pmc2 ok" &&
bash tools/gpu_pmc.sh "${1:-round}/pmc2s" --config 2 --op sha1 > /dev/null && echo "pmc2s ok" &&
bash tools/gpu_pmc.sh "${1:-round}/pmc3" --config 3 > /dev/null && echo "pmc3 ok" &&
bash tools/gpu_pmc.sh "${1:-round}/pmc4" --config 4 > /dev/null && echo "pmc4 ok" &&
bash tools/gpu_pmc.sh "${1:-round}/pmc_rc4" --op rc4 > /dev/null && echo "pmc rc4 ok" &&
bash tools/gpu_pmc.sh "${1:-round}/pmc_rc4md5" --op rc4md5 > /dev/null && echo "pmc rc4md5 ok" &&
bash tools/gpu_pmc.sh "${1:-round}/pmc_md" --op metadata > /dev/null && echo "pmc metadata ok" &&
bash tools/gpu_pmc.sh "${1:-round}/pmc_seg" --op md5seg > /dev/null && echo "pmc md5seg ok" &&
bash tools/gpu_pmc.sh "${1:-round}/pmc_b64" --op base64 > /dev/null && echo "pmc base64 ok"
rc=$?
tail -3 "$OUT/pytest_gpu.log"
exit $rc
