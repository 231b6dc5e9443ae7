#!/bin/bash
# Round 6: the line kernel's first line pair issued before the workgroup barrier (product) against
# barrier-first (tools/mb/line_ab_bf, -DBRB_LINE_BARRIER_FIRST), alternating processes, cfg2 and
# the cfg5 shard; parity of the product's line shapes; then one PMC pass over tools/mb/line_ab
# (round-5 vs round-6 kernel: VALU / SALU / LDS instructions per launch).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06d}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_all_devices.py \
    -k "line_kernel or cfg5_full or cfg2_full or large_batch or many_groups or edge_lengths or unaligned or line_forced or golden_edge" \
    > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for b in line_ab line_ab_bf; do
    timeout -k 10 120 tools/mb/$b 65536 1500 3 400 > $O/cfg2_${b}_$r.txt 2>&1 || { tail -3 $O/cfg2_${b}_$r.txt; exit 1; }
    echo "cfg2 $b $r: $(grep MEDIAN $O/cfg2_${b}_$r.txt | tr '\n' ' ')"
    timeout -k 10 200 tools/mb/$b 1048576 1500 3 40 > $O/cfg5_${b}_$r.txt 2>&1 || { tail -3 $O/cfg5_${b}_$r.txt; exit 1; }
    echo "cfg5 $b $r: $(grep MEDIAN $O/cfg5_${b}_$r.txt | tr '\n' ' ')"
  done
done
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD \
    --kernel-trace --output-format csv -d $O/pmc_line_ab -o run -- tools/mb/line_ab 1048576 1500 1 5 > $O/pmc_line_ab.log 2>&1 || { tail -5 $O/pmc_line_ab.log; exit 1; }
python3 tools/pmc_summary.py $O/pmc_line_ab "digest_line_kernel<AlgLit, 8, true, true>" > $O/pmc_line_r06.txt
python3 tools/pmc_summary.py $O/pmc_line_ab "digest_line_kernel<AlgLit, 8, true, true, true" > $O/pmc_line_r05.txt
head -30 $O/pmc_line_r05.txt $O/pmc_line_r06.txt
