#!/bin/bash
# SQ counter passes (one rocprofv3 run per group, kernel-trace only) over an
# arbitrary python command; prints per-kernel means for kernels matching $1.
#   tools/pmc_cmd.sh k_walk tools/grid_bin_case.py --reps 2 --ranges 0-15
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
pat=$1; shift
out=gpurun_out/pmc_$pat
mkdir -p $out
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_INSTS_SMEM" \
           "SQ_IFETCH SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $out -o p$i \
        -- python3 "$@" > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; exit 1; }
done
python3 tools/pmc_table.py $out $pat
