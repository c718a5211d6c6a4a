#!/bin/bash
# Round-4 walk iteration: the walk's GPU tests with the flat walk, then the
# rocprof A/B (tools/walk_ab.sh).  Stops at the first crash / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DFHIP_WALK_FLAT=${FLAT:-1} timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    ${TESTS:-tests/test_gpu_encoders.py tests/test_gpu_step_structures.py tests/test_gpu_native_step.py tests/test_gpu_shading.py tests/test_gpu_bf16.py} \
    > gpurun_out/t_walk.log 2>&1
rc=$?
tail -5 gpurun_out/t_walk.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
bash tools/walk_ab.sh > gpurun_out/walk_ab.txt 2>&1
rc=$?
cat gpurun_out/walk_ab.txt
exit $rc
