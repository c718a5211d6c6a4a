#!/bin/bash
# Iteration session: given pytest files ($TESTS), then a graph bench line and a
# rocprofv3 kernel-stats pass.  Stops at the first crash / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TESTS=${TESTS:-tests}
timeout -k 10 500 python -m pytest $TESTS -q -x -p no:cacheprovider -m gpu > gpurun_out/pt_iter.log 2>&1
rc=$?
tail -12 gpurun_out/pt_iter.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/bench_graph.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_graph.log; exit 3; }
tail -1 gpurun_out/bench_graph.log | cut -c1-700
bash tools/gpu_prof.sh > /dev/null 2>&1 || { echo "prof failed"; exit 4; }
python3 tools/prof_top.py gpurun_out/prof/run_kernel_stats.csv 14
exit $rc
