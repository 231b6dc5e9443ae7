#!/bin/bash
# Segment / MetaData line-staged kernels (round 4): parity tests, then interleaved A/B of the bench
# lines (test option seg_line 1 = line-staged, 0 = per-lane), then a kernel-trace profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-seg}
OPS=${2:-md5seg}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_segments.py tests/test_metadata.py -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for r in 1 2; do
  for op in $OPS; do
    for v in 1 0; do
      timeout -k 10 120 python bench.py --op $op --no-cpu-baseline --test-option seg_line=$v > "$OUT/b_${op}_${v}_$r.json" 2> "$OUT/b_${op}_${v}_$r.err" || { echo "bench $op $v failed"; tail -5 "$OUT/b_${op}_${v}_$r.err"; exit 1; }
      python -c "import json,sys; d=json.load(open('$OUT/b_${op}_${v}_$r.json')); print('$op seg_line=$v', d['roofline']['launch_us_avg'], 'us', d['roofline']['frac'])"
    done
  done
done
for op in $OPS; do
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$op" -o run --output-format csv -- \
    python3 bench.py --op $op --no-cpu-baseline > "$OUT/prof_$op.json" 2> "$OUT/prof_$op.err" || { echo "rocprof failed"; exit 1; }
done
echo done
