#!/bin/bash
# Round-5 A/B: the stencil field forward sharing the centre's coarse-level
# corner quads (default library) against lib/libdfhip_noshare.so
# (DFHIP_FWD_SHARE=0) and the probe libraries (DFHIP_FWD_SHARE_PROBE).  Field +
# shading tests on the default library, then per library rocprofv3 kernel
# stats of the textureless step (and of the C2 steps for the default).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab2}
mkdir -p $OUT
L=$PWD/single-stable-dreamfusion_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_field.py tests/test_gpu_shading.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    > $OUT/pytest_base.log 2>&1 || { echo "pytest base failed"; tail -30 $OUT/pytest_base.log; exit 1; }
tail -1 $OUT/pytest_base.log
for v in ${VARS:-base noshare}; do
  if [ $v = base ]; then unset DFHIP_LIB; else export DFHIP_LIB=$L/libdfhip_$v.so; fi
  echo "=== $v"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/shade_$v -o run \
      -- python tools/shade_steps.py textureless 30 > $OUT/shade_$v.log 2>&1 \
      || { echo "shade $v failed"; tail -20 $OUT/shade_$v.log; exit 3; }
  python tools/prof_top.py $OUT/shade_$v/run_kernel_stats.csv 6
  if [ $v = base ]; then TAG=${v}_ab2 TOPN=6 bash tools/prof_c2.sh || exit 4; fi
done
