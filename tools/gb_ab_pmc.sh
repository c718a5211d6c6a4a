#!/bin/bash
# PMC (one counter group per rocprofv3 run) of the windowed vs slice walk on a level range.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
r=${1:-0-15}
for mode in win slices; do
    out=gpurun_out/gbpmc/$mode$r
    mkdir -p $out
    if [ $mode = slices ]; then export DFHIP_GRID_NOWIN=1; fi
    i=0
    for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY" \
               "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"; do
        i=$((i+1))
        timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $out -o p$i \
            -- python3 tools/grid_bin_case.py --reps 2 --ranges $r > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $out/p$i.log; exit 1; }
    done
    echo "== $mode $r"
    python3 tools/pmc_table.py $out walk
done
