#!/bin/bash
# PMC passes over the grid backward case for a given walk switch ($DBG).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/walkpmc${DBG:-0}
mkdir -p $out
i=0
for grp in "TA_BUSY_avr TA_BUSY_max TCP_TOTAL_CACHE_ACCESSES_sum TD_BUSY_avr" \
           "TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $out -o p$i \
        -- python3 tools/walk_trace.py --reps 1 --dbg ${DBG:-0} > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; }
done
python3 tools/pmc_table.py $out k_walk
