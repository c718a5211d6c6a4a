#!/bin/bash
# The walk's two launch-sequence states (round 6: 182 vs 217 us): SQ / GRBM /
# TCC counters of k_walk with the kept-clean scratch (fast) and with the
# per-step fill ahead of the binning (DFHIP_KEPT_CLEAN=0, slow), one
# rocprofv3 run per counter group and variant, each under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
F="--no-cpu-baseline --no-kernel-timing --no-alt-backward --no-shading --no-infer --no-traffic --no-c5 --no-module-path"
for v in 1 0; do
  out=gpurun_out/${1:-pmc_walk}/kc$v
  mkdir -p $out
  export DFHIP_KEPT_CLEAN=$v
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
             "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $out -o p$i \
        -- python3 bench.py --steps 20 --warmup 10 $F > $out/p$i.log 2>&1 || { echo "pass $v/$i failed"; tail -5 $out/p$i.log; exit 2; }
  done
  echo "== kept_clean=$v"
  python3 tools/pmc_table.py $out k_walkIDF
  python3 tools/pmc_table.py $out k_bin_fast
done
