#!/bin/bash
# MFMA counters of the train-step field kernels and the C4 renderer: one
# rocprofv3 pass (kernel-trace only) over a short bench run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/pmcmfma
mkdir -p $out
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d $out -o p1 \
    -- python3 bench.py --steps 4 --warmup 3 --no-cpu-baseline --no-kernel-timing --no-alt-backward --no-shading --infer-res 800 \
    > $out/p1.log 2>&1 || { echo "pmc pass failed"; tail -5 $out/p1.log; exit 1; }
python3 tools/pmc_mfma_summary.py $out
