#!/bin/bash
# PMC passes (one rocprofv3 --pmc pass per counter group; kernel-trace only, no sys/runtime trace).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc}
shift
ARGS="${@:---config 2}"
mkdir -p "$OUT"
[ -f "$OUT/counters.txt" ] || timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES" \
           "GRBM_GUI_ACTIVE GRBM_COUNT FETCH_SIZE" "WRITE_SIZE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES" \
           "TA_BUSY_avr TA_TA_BUSY_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- \
      python3 bench.py $ARGS --no-cpu-baseline --no-pcie --no-cfg5 --steps 10 --warmup 2 --settle-s 0 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
ls "$OUT"
