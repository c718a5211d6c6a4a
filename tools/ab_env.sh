#!/bin/bash
# A/B of an environment switch on the C2 bench line, interleaved A B A B:
#   VAR=DFHIP_MARCH_ORDER A=0 B=1 bash tools/ab_env.sh
# prints ms/step and the named kernel regions of each run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VAR=${VAR:?} A=${A:?} B=${B:?} REGIONS=${REGIONS:-march_rays_train_count,grid_encode_backward}
ARGS="--steps 40 --warmup 10 --no-cpu-baseline --no-traffic --no-infer --no-c5 --no-module-path --no-shading --no-alt-backward ${BENCH_ARGS:-}"
for rep in 1 2; do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 300 python bench.py $ARGS > gpurun_out/ab_$v.log 2>&1 \
      || { echo "bench $VAR=$v failed"; tail -20 gpurun_out/ab_$v.log; exit 3; }
    python - "$v" "$REGIONS" <<'EOF'
import json, sys
d = json.loads([l for l in open(f"gpurun_out/ab_{sys.argv[1]}.log") if l.startswith("{")][-1])
k = d.get("kernels", {})
regs = " ".join(f"{r} {k[r]['avg_us']}" for r in sys.argv[2].split(",") if r in k)
print(f"{sys.argv[1]}: {d['ms_per_step']} ms/step host {d['host_issue_ms_per_step']} | {regs}")
EOF
  done
done
