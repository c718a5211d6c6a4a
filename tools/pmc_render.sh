#!/bin/bash
# C4 renderer counters: the SQ / TA / TCP / TCC groups of tools/pmc_step.sh
# (one rocprofv3 run per group, kernel trace only, each under its own time
# limit) over tools/infer_case.py (the bench's 800x800 frame), then the
# per-wave phase cycles (dfhip_render_rays_infer_prof).  Says how busy the
# SIMDs already are, i.e. what a producer / consumer wave split could add.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${TAG:-pmc_render}
mkdir -p $out
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA TA_BUSY_avr TA_BUSY_max TD_BUSY_avr" \
           "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $out -o p$i \
        -- python3 tools/infer_case.py --reps 3 > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; exit 2; }
done
python3 tools/pmc_table.py $out k_render_infer
timeout -k 10 120 python3 tools/infer_case.py --reps 3 --profile > $out/phases.log 2>&1 || { echo "phases failed"; tail -5 $out/phases.log; exit 3; }
tail -3 $out/phases.log
