#!/bin/bash
# A/B of an environment switch on the C4 inference legs (grid R0 and sphere
# R1), interleaved: VAR=DFHIP_COARSE A=0 B=1 bash tools/infer_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VAR=${VAR:?} A=${A:?} B=${B:?}
ARGS="--steps 2 --warmup 2 --no-cpu-baseline --no-traffic --no-c5 --no-module-path --no-shading --no-alt-backward --no-kernel-timing"
for rep in 1 2; do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 300 python bench.py $ARGS > gpurun_out/iab_$v.log 2>&1 \
      || { echo "bench $VAR=$v failed"; tail -20 gpurun_out/iab_$v.log; exit 3; }
    python - "$v" <<'PY'
import json, sys
d = json.loads([l for l in open(f"gpurun_out/iab_{sys.argv[1]}.log") if l.startswith("{")][-1])
for key in ("inference", "inference_sphere"):
    i = d.get(key, {})
    print(f"{sys.argv[1]} {key}: {i.get('ms_per_frame')} ms/frame, kernel {i.get('kernel_avg_us')} us, "
          f"{i.get('samples_per_frame')} samples, {i.get('samples_per_sec', 0) / 1e9:.2f} G/s, "
          f"loop {i.get('loop_ms_per_frame')} ms ({i.get('speedup_vs_loop')}x)")
PY
  done
done
