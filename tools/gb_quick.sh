#!/bin/bash
# Grid-backward iteration: binned-backward GPU tests, the full-range timing on
# a real 128x128 march, one bench line (C2 only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/gbq
timeout -k 10 300 python -u -m pytest tests/test_gpu_encoders.py tests/test_gpu_field_oracle.py tests/test_gpu_native_step.py -x -q -p no:cacheprovider -m gpu -k "binned or native or chain" --timeout 120 --timeout-method thread > gpurun_out/gbq/pt.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/gbq/pt.log; exit 1; }
tail -1 gpurun_out/gbq/pt.log
timeout -k 10 200 python tools/grid_bin_case.py --reps 10 --ranges ${RANGES:-0-15,0-2,3-8,9-15} || exit 2
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-alt-backward --no-shading --no-infer --no-traffic --no-c5 --no-module-path > gpurun_out/gbq/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/gbq/bench.log; exit 3; }
python -c "import json; d=json.loads([l for l in open('gpurun_out/gbq/bench.log') if l.startswith('{')][-1]); print('ms/step', d['ms_per_step'], 'gb_us', d['kernels']['grid_encode_backward']['avg_us'])"
