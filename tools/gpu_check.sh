#!/bin/bash
# One GPU session: parity tests, smoke, bench.  Stops at the first crash /
# timeout (exit codes other than 0/1 from pytest), never retries.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-30}
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 "$@" \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
src=$?
tail -3 gpurun_out/smoke.log
if [ $src -ne 0 ]; then echo "smoke failed rc=$src"; exit $src; fi
timeout -k 10 600 python bench.py --steps $STEPS --warmup 10 > gpurun_out/bench.log 2>&1
brc=$?
tail -2 gpurun_out/bench.log
exit $(( rc > brc ? rc : brc ))
