#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run (separate from PMC passes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
STEPS=${STEPS:-20}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run \
    -- python bench.py --steps $STEPS --warmup 5 --no-cpu-baseline --no-kernel-timing \
    > gpurun_out/prof/bench_prof.log 2>&1
rc=$?
tail -2 gpurun_out/prof/bench_prof.log
find gpurun_out/prof -name "*stats*" | head
exit $rc
