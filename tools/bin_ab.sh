#!/bin/bash
# Binning A/B: the default library against lib/libdfhip_${VAR:-ballot}.so —
# the encoder GPU tests with the variant, then rocprofv3 kernel stats of the
# albedo bin case and of textureless steps with each, and the bin kernels'
# LDS counters (SQ_ACTIVE_INST_LDS, SQ_LDS_BANK_CONFLICT) with each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-bin_ab}
mkdir -p $OUT
VLIB=$PWD/single-stable-dreamfusion_amd/lib/libdfhip_${VAR:-ballot}.so
DFHIP_LIB=$VLIB timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_encoders.py} -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in base var; do
  if [ $v = base ]; then unset DFHIP_LIB; else export DFHIP_LIB=$VLIB; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/case_$v -o run \
      -- python tools/grid_bin_case.py --modes 0 --ranges 0-15 --reps 5 > $OUT/case_$v.log 2>&1 \
      || { echo "case $v failed"; tail -20 $OUT/case_$v.log; exit 2; }
  echo "=== albedo case $v"; grep median $OUT/case_$v.log; python tools/prof_top.py $OUT/case_$v/run_kernel_stats.csv 3
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/shade_$v -o run \
      -- python tools/shade_steps.py textureless 30 > $OUT/shade_$v.log 2>&1 \
      || { echo "shade $v failed"; tail -20 $OUT/shade_$v.log; exit 3; }
  echo "=== textureless $v"; python tools/prof_top.py $OUT/shade_$v/run_kernel_stats.csv 8
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_INSTS_VALU \
      --output-format csv -d $OUT/pmc_$v -o p1 -- python3 tools/shade_steps.py textureless 6 > $OUT/pmc_$v.log 2>&1 \
      || { echo "pmc $v failed"; tail -5 $OUT/pmc_$v.log; exit 4; }
  for k in k_bin_fast k_walk_flat; do python3 tools/pmc_table.py $OUT/pmc_$v $k; done
done
