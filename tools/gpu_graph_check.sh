#!/bin/bash
# Graph-step session: new graph tests + network tests, then eager and graph bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_graph.py tests/test_gpu_network.py tests/test_gpu_raymarching.py -q -p no:cacheprovider --timeout 300 -x \
    > gpurun_out/pytest_graph.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_graph.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/bench_graph.log 2>&1 || { echo "graph bench failed"; tail -30 gpurun_out/bench_graph.log; exit 3; }
tail -1 gpurun_out/bench_graph.log
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --eager > gpurun_out/bench_eager.log 2>&1 || { echo "eager bench failed"; tail -30 gpurun_out/bench_eager.log; exit 3; }
tail -1 gpurun_out/bench_eager.log
exit $rc
