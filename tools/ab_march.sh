#!/bin/bash
# March-count A/B: bit-exact march tests on the new library, then rocprof
# kernel stats of the C2 headline for lib/libdfhip_base.so and lib/libdfhip.so
# (two alternating pairs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/abm
timeout -k 10 300 python -u -m pytest tests/test_gpu_raymarching.py tests/test_gpu_field_oracle.py tests/test_golden.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    > gpurun_out/abm/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/abm/pytest.log; exit 1; }
tail -1 gpurun_out/abm/pytest.log
for i in 1 2; do
  DFHIP_LIB=single-stable-dreamfusion_amd/lib/libdfhip_base.so TAG=base$i STEPS=40 TOPN=12 bash tools/prof_c2.sh > gpurun_out/abm/base$i.txt || exit 2
  TAG=new$i STEPS=40 TOPN=12 bash tools/prof_c2.sh > gpurun_out/abm/new$i.txt || exit 3
done
grep -H "march_train_count\|k_march_train_emit" gpurun_out/abm/*.txt
grep -H -o '"ms_per_step": [0-9.]*' gpurun_out/prof_*/bench.log
