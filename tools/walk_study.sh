#!/bin/bash
# Grid-backward study: per-level-range timings of the binned backward on a
# real 128x128 march, LDS atomic micro-benchmark, then PMC passes (one
# rocprofv3 run per counter group) over the full-range case.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/walk
mkdir -p $out
timeout -k 10 120 python tools/grid_bin_case.py --reps 10 --ranges 0-15,0-2,3-8,9-15 > $out/ranges.log 2>&1 || { echo "ranges failed"; tail $out/ranges.log; exit 1; }
cat $out/ranges.log
if [ -x tools/micro/lds_atomic ]; then timeout -k 5 60 tools/micro/lds_atomic > $out/lds_atomic.log 2>&1; cat $out/lds_atomic.log; fi
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $out -o p$i \
        -- python3 tools/grid_bin_case.py --reps 2 --ranges 0-15 > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; exit 2; }
done
python3 tools/pmc_table.py $out gb
