# bench.py C4 legs (R0, R1) with the background net beside the render vs after
# it (DFHIP_INFER_OVERLAP_BG=0), alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06y
mkdir -p $O
F="--steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing --no-alt-backward --no-shading --no-traffic --no-c5 --no-module-path"
for i in 1 2; do
  for v in 1 0; do
    DFHIP_INFER_OVERLAP_BG=$v timeout -k 10 300 python -u $R/bench.py $F > $O/b$v$i.log 2>&1 || exit 1
    python - $O/b$v$i.log $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("overlap", sys.argv[2], *[(k, d[k]["ms_per_frame"], d[k]["kernel_avg_us"]) for k in ("inference", "inference_sphere")])
PY
  done
done
