#!/bin/bash
# Quick GPU iteration: the given test files, then one bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TESTS=${TESTS:-tests}
timeout -k 10 400 python -u -m pytest $TESTS -x -v -p no:cacheprovider -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt_quick.log 2>&1
rc=$?
tail -15 gpurun_out/pt_quick.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_quick.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_quick.log; exit 3; }
tail -1 gpurun_out/bench_quick.log
