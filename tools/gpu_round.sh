#!/bin/bash
# Full round check: GPU parity tests, smoke, a default bench line, and a
# rocprofv3 kernel-stats pass of a short bench.  Each GPU step has its own
# time limit; the script stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-round}
mkdir -p $OUT
# SKIP_TESTS=1: the bench and profiles only (tests and smoke green on this tree)
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread --durations=30 \
    > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
    || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 2; }
tail -1 $OUT/smoke.log
fi
timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1 \
    || { echo "bench failed"; tail -30 $OUT/bench.log; exit 3; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
python -c "import json; d=json.load(open('$OUT/bench.json')); print('ms/step', d['ms_per_step'], 'value', d['value'], 'roof', d.get('roofline',{}).get('frac'), 'infer', d.get('inference',{}).get('ms_per_frame'))"
# the same child command bench.py's roofline passes profile: its kernel trace
# reproduces the line's roofline.frac (tools/roofline_check.py)
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run \
    -- python bench.py --steps 16 --warmup ${CHILD_WARMUP:-34} --no-cpu-baseline --no-kernel-timing --no-alt-backward \
       --no-shading --no-infer --no-traffic --no-c5 --no-module-path \
    > $OUT/bench_prof.log 2>&1 || { echo "prof failed"; tail -20 $OUT/bench_prof.log; exit 4; }
python tools/prof_top.py $OUT/prof/run_kernel_stats.csv 25 > $OUT/rocprof_top.txt
cat $OUT/rocprof_top.txt
python tools/roofline_check.py $OUT/bench.json $OUT/prof/run_kernel_trace.csv | tee $OUT/roofline_check.json
# the textureless step's kernels (the shaded steps' profile)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/shprof -o run \
    -- python tools/shade_steps.py textureless 30 > $OUT/shade_prof.log 2>&1 \
    || { echo "shade prof failed"; tail -20 $OUT/shade_prof.log; exit 5; }
python tools/prof_top.py $OUT/shprof/run_kernel_stats.csv 25 > $OUT/rocprof_shade_top.txt
head -8 $OUT/rocprof_shade_top.txt
# the shading roofline's child (bench.py --shade textureless): its trace
# reproduces shading.roofline.frac
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/shchild -o run \
    -- python bench.py --steps 16 --warmup ${CHILD_WARMUP:-34} --no-cpu-baseline --no-kernel-timing --no-alt-backward \
       --no-shading --no-infer --no-traffic --no-c5 --no-module-path --shade textureless \
    > $OUT/shchild.log 2>&1 || { echo "shade child prof failed"; tail -20 $OUT/shchild.log; exit 6; }
python tools/roofline_check.py $OUT/bench.json $OUT/shchild/run_kernel_trace.csv --shading | tee $OUT/roofline_check_shading.json
