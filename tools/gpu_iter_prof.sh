#!/bin/bash
# Iteration loop: the given GPU test files, then a rocprofv3 kernel-trace of a
# short bench run, summarised to gpurun_out/prof/top.txt.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TESTS=${TESTS:-tests}
timeout -k 10 400 python -u -m pytest $TESTS -x -q -p no:cacheprovider -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt_iter.log 2>&1
rc=$?
tail -5 gpurun_out/pt_iter.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run \
    -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing ${BENCH_ARGS:-} \
    > gpurun_out/prof/bench_prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof/bench_prof.log; exit 3; }
grep '^{' gpurun_out/prof/bench_prof.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/step', d['ms_per_step'], 'infer ms', d.get('inference',{}).get('ms_per_frame'))"
python tools/prof_top.py gpurun_out/prof/run_kernel_stats.csv 25 > gpurun_out/prof/top.txt
cat gpurun_out/prof/top.txt
