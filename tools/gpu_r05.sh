#!/bin/bash
# Round-5 iteration: GPU tests (TESTS, default all), then one short bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05}
mkdir -p $OUT
timeout -k 10 ${PT_LIMIT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread --durations=15 \
    > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
if [ -n "${NO_BENCH:-}" ]; then exit 0; fi
timeout -k 10 400 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench.log 2>&1 \
    || { echo "bench failed"; tail -30 $OUT/bench.log; exit 3; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
python -c "import json; d=json.load(open('$OUT/bench.json')); print('ms/step', d['ms_per_step'], 'value', d['value'], 'roof', d.get('roofline',{}).get('frac'), 'shade', {k: d.get('shading',{}).get(k) for k in ('textureless_ms_per_step','iters_weighted_ms_per_step')}, 'infer', d.get('inference',{}).get('ms_per_frame'))"
