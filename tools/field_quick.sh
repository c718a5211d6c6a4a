#!/bin/bash
# Field-kernel iteration: the field / encoder / render / native-step GPU tests,
# then one bench line with the C4 frame.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fq
timeout -k 10 500 python -u -m pytest tests/test_gpu_field.py tests/test_gpu_field_oracle.py tests/test_gpu_render.py tests/test_gpu_native_step.py tests/test_gpu_bf16.py tests/test_gpu_encoders.py -x -q -p no:cacheprovider -m gpu --timeout 180 --timeout-method thread > gpurun_out/fq/pt.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/fq/pt.log; exit 1; }
tail -1 gpurun_out/fq/pt.log
timeout -k 10 400 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-alt-backward --no-shading --no-traffic > gpurun_out/fq/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/fq/bench.log; exit 3; }
python - <<'PY'
import json
d = json.loads([l for l in open('gpurun_out/fq/bench.log') if l.startswith('{')][-1])
fm = d['field_mlp']
print('ms/step', d['ms_per_step'], 'fwd_us', fm['forward']['avg_us'], 'rows', fm['rows'],
      'infer_ms', d['inference']['ms_per_frame'], 'c5_ms', d['c5']['ms_per_step'])
PY
