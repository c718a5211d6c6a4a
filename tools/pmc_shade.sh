#!/bin/bash
# SQ / TA / TCP / TCC counter passes (one rocprofv3 run per group, kernel
# trace only, each under its own time limit) over six textureless steps; prints
# per-kernel means for the step's main kernels (tools/pmc_table.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${TAG:-pmc_shade}
mkdir -p $out
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA TA_BUSY_avr TA_BUSY_max TD_BUSY_avr" \
           "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $out -o p$i \
        -- python3 tools/shade_steps.py textureless 6 > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; exit 2; }
done
for k in k_walk_flat k_field_bwd k_field_fwd_fused k_bin_fast k_stencil; do
    python3 tools/pmc_table.py $out $k
done
