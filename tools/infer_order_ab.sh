#!/bin/bash
# C4 queue order A/B: pixel order (DFHIP_INFER_ORDER=0) against the native
# chunk order (dfhip_render_ray_order) at chunks of 2^5 / 2^6 / 2^7 rays; the
# renderer tests first, then per setting the frame time and the drain profile
# (R0 grid occupancy and the R1 sphere).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-order}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_render.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    > $OUT/pytest_render.log 2>&1 || { echo "pytest render failed"; tail -30 $OUT/pytest_render.log; exit 1; }
tail -1 $OUT/pytest_render.log
for s in ${SETS:-0:6 1:5 1:6 1:7}; do
  o=${s%%:*}; cl=${s#*:}
  for sph in "" "--sphere"; do
    DFHIP_INFER_ORDER=$o DFHIP_INFER_CHUNK_LOG2=$cl timeout -k 10 120 python3 tools/infer_case.py --reps 10 --profile $sph > $OUT/o${o}_${cl}${sph}.log 2>&1 \
        || { echo "order $s failed"; tail -5 $OUT/o${o}_${cl}${sph}.log; exit 2; }
    echo "=== order $o chunk 2^$cl $sph"; tail -3 $OUT/o${o}_${cl}${sph}.log
  done
done
