# C4 renderer: deeper lookahead when every marching lane of the wave skipped
# last time (-DDFHIP_RENDER_AHEAD_DEEP=K builds as lib/libdfhip_d{4,8}.so; the
# option was removed after this A/B) vs K = 2 throughout: render tests with d8,
# then tools/infer_case.py interleaved
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
L=$R/single-stable-dreamfusion_amd/lib
mkdir -p gpurun_out
DFHIP_LIB=$L/libdfhip_d8.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_render.py > gpurun_out/r06u_test.txt 2>&1
tail -1 gpurun_out/r06u_test.txt
for sc in "" "--sphere"; do
  for i in 1 2 3; do
    for v in base d4 d8; do
      if [ $v = base ]; then unset DFHIP_LIB; else export DFHIP_LIB=$L/libdfhip_$v.so; fi
      echo "== $v $sc"; timeout -k 10 180 python -u $R/tools/infer_case.py $sc | grep res=
    done
  done
done
