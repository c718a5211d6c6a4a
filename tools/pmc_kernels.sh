#!/bin/bash
# SQ / TCC counter passes (one rocprofv3 run per group, kernel-trace only) over
# tools/bench_kernels.py --only $1; prints per-kernel means (tools/pmc_table.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
only=$1
out=gpurun_out/pmck_$only
mkdir -p $out
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_INSTS_MFMA" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA" \
           "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $out -o p$i \
        -- python3 tools/bench_kernels.py --only $only --reps 2 > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; }
done
python3 tools/pmc_table.py $out $only
