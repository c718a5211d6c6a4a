# bench.py C4 legs after the other legs: which earlier leg slows the R1 frame
# (C4 alone vs with C5 / the shading legs; then the module path, the kernel
# timing and alternative backward, the traffic passes)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06af
mkdir -p $O
BASE="--steps 10 --warmup 5 --no-cpu-baseline --no-shading --no-c5"
run() {
  local tag=$1; shift
  timeout -k 10 400 python -u $R/bench.py "$@" > $O/$tag.log 2>&1 || exit 1
  python - $O/$tag.log $tag <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], *[(k, d[k]["ms_per_frame"], d[k]["kernel_avg_us"]) for k in ("inference", "inference_sphere")])
PY
}
run alone $BASE --no-kernel-timing --no-alt-backward --no-traffic --no-module-path
run module $BASE --no-kernel-timing --no-alt-backward --no-traffic
run timing_alt $BASE --no-traffic --no-module-path
run traffic $BASE --no-kernel-timing --no-alt-backward --no-module-path
