# the full default bench.py with the background net beside the C4 render (the
# render and the net on a consecutive pair of pool streams) or after it
# (DFHIP_INFER_OVERLAP_BG=0): render tests, then the C4 legs at the end of the full run
# (runs of this script: main + one side stream; paired streams with the net after the
# order; paired streams with the net from before the order: profiles/r06/c4_bg_overlap_ab.txt)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ag
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_render.py > $O/test.txt 2>&1 || exit 1
tail -1 $O/test.txt
for v in 1 0; do
  DFHIP_INFER_OVERLAP_BG=$v timeout -k 10 600 python -u $R/bench.py --no-cpu-baseline > $O/b$v.log 2>&1 || exit 1
  python - $O/b$v.log $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("overlap", sys.argv[2], d["ms_per_step"], *[(k, d[k]["ms_per_frame"], d[k]["kernel_avg_us"], d[k]["order_avg_us"]) for k in ("inference", "inference_sphere")])
PY
done
