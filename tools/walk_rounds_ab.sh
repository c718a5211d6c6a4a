#!/bin/bash
# Flat-walk rounds A/B (DFHIP_WALK_QR: the stencil walk takes its chunk in
# windows of ~1024 x QR entries; qr8s: a workgroup barrier between rounds):
# the binned / stencil encoder tests on qr8, then per library the textureless
# step's kernels (rocprofv3 stats), then the C4 renderer's drain profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-wr}
mkdir -p $OUT
L=$PWD/single-stable-dreamfusion_amd/lib
DFHIP_LIB=$L/libdfhip_qr8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_encoders.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "binned or stencil or walk" \
    > $OUT/pytest_qr8.log 2>&1 || { echo "pytest qr8 failed"; tail -30 $OUT/pytest_qr8.log; exit 1; }
tail -1 $OUT/pytest_qr8.log
for v in ${VARS:-base qr4 qr8 qr16 qr8s}; do
  if [ $v = base ]; then unset DFHIP_LIB; else export DFHIP_LIB=$L/libdfhip_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/shade_$v -o run \
      -- python tools/shade_steps.py textureless 30 > $OUT/shade_$v.log 2>&1 \
      || { echo "shade $v failed"; tail -20 $OUT/shade_$v.log; exit 3; }
  echo "=== $v"; python tools/prof_top.py $OUT/shade_$v/run_kernel_stats.csv 3
done
unset DFHIP_LIB
timeout -k 10 120 python3 tools/infer_case.py --reps 3 --profile > $OUT/phases.log 2>&1 || { echo "phases failed"; tail -5 $OUT/phases.log; exit 4; }
tail -3 $OUT/phases.log
