#!/bin/bash
# stencil-group binning: parity tests, then the shaded-step bench legs A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_encoders.py tests/test_gpu_shading.py tests/test_gpu_bf16.py -x -q -m gpu -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/pt_c.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pt_c.log; exit 1; }
tail -2 gpurun_out/pt_c.log
for v in 0 1 0 1; do
  DFHIP_STENCIL_BIN=$v timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-traffic --no-infer --no-c5 --no-module-path --no-alt-backward --no-kernel-timing > gpurun_out/sb_$v.log 2>&1 || { echo "bench failed"; tail gpurun_out/sb_$v.log; exit 2; }
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/sb_$v.log') if l.startswith('{')][-1]); print('$v', d['ms_per_step'], d['shading'])"
done
