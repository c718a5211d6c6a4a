#!/bin/bash
# Walk A/B by rocprofv3 kernel stats: the C2 headline and the textureless
# step, each with the default walk form of a variant library built with
# -DDFHIP_WALK_MODE_DEFAULT=v (1 flat walk, 0 per-segment walk, 2 per-wave).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in ${VALS:-2 1 0}; do
  lib=$(bash tools/variant_lib.sh flat$v gridbin.hip "-DDFHIP_WALK_MODE_DEFAULT=$v" | tail -1) || exit 4
  export DFHIP_LIB=$PWD/$lib
  TAG=flat$v TOPN=12 bash tools/prof_c2.sh || exit 4
  OUT=gpurun_out/prof_shade_flat$v
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run \
      -- python tools/shade_steps.py textureless 30 > $OUT/log.txt 2>&1 || { echo "shade prof failed"; tail -5 $OUT/log.txt; exit 4; }
  python tools/prof_top.py $OUT/run_kernel_stats.csv 8 > $OUT/top.txt
  cat $OUT/top.txt
done
