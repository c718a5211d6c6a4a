# C4 renderer: K-cell lookahead in the per-lane march (lib/libdfhip_a{2,3}.so; K = 4 measured first
# built with -DDFHIP_RENDER_AHEAD=K) vs K = 1: render tests with K = 3, then
# tools/infer_case.py R0 / R1 interleaved
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
L=$R/single-stable-dreamfusion_amd/lib
mkdir -p gpurun_out
DFHIP_LIB=$L/libdfhip_a3.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_render.py > gpurun_out/r06s_test.txt 2>&1
tail -1 gpurun_out/r06s_test.txt
for sc in "" "--sphere"; do
  for i in 1 2 3; do
    for v in base a2 a3; do
      if [ $v = base ]; then unset DFHIP_LIB; else export DFHIP_LIB=$L/libdfhip_$v.so; fi
      echo "== $v $sc"; timeout -k 10 180 python -u $R/tools/infer_case.py $sc | grep res=
    done
  done
done
