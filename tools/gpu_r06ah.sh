# after the background-launch refactor: render tests and the C4 legs once
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ah
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_render.py > $O/test.txt 2>&1 || exit 1
tail -1 $O/test.txt
timeout -k 10 300 python -u $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing --no-alt-backward --no-shading --no-traffic --no-c5 --no-module-path > $O/b.log 2>&1 || exit 1
python - $O/b.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(*[(k, d[k]["ms_per_frame"], d[k]["kernel_avg_us"]) for k in ("inference", "inference_sphere")])
PY
