# cooperative drain of the C4 renderer: its tests, then the C4 leg of the
# bench with DFHIP_INFER_COOP 0 / 8 / 32 / 64, interleaved twice
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06m}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_render.py -m gpu -x -v --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
F="--no-cpu-baseline --no-kernel-timing --no-alt-backward --no-shading --no-traffic --no-c5 --no-module-path --steps 5 --warmup 3"
for rep in 1 2; do
  for v in 0 8 32 64; do
    export DFHIP_INFER_COOP=$v
    timeout -k 10 300 python bench.py $F > $O/c4_$v.$rep.log 2>&1 || exit 1
    python - $O/c4_$v.$rep.log $v <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
inf = json.loads(line)["inference"]
r1 = inf.get("r1", inf.get("sphere", {}))
print("coop", sys.argv[2], "R0 ms/frame", inf["ms_per_frame"], "kernel us", inf.get("kernel_avg_us"), "G/s", round(inf["samples_per_sec"] / 1e9, 3), "| R1", {k: r1.get(k) for k in ("ms_per_frame", "kernel_avg_us", "samples_per_sec")} if isinstance(r1, dict) else r1)
PY
  done
done
