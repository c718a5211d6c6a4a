# C4: samples per round (kBatch 64 / 96 / 128: -DDFHIP_RENDER_BATCH builds as
# lib/libdfhip_b{96,128}.so, removed after this A/B) on the final layout;
# render tests with 128, then infer_case R0 / R1 interleaved
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
L=$R/single-stable-dreamfusion_amd/lib
DFHIP_LIB=$L/libdfhip_b128.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_render.py > gpurun_out/r06ac_test.txt 2>&1
tail -1 gpurun_out/r06ac_test.txt
for sc in "" "--sphere"; do
  for i in 1 2 3; do
    for v in base b96 b128; do
      if [ $v = base ]; then unset DFHIP_LIB; else export DFHIP_LIB=$L/libdfhip_$v.so; fi
      echo "== $v $sc"; timeout -k 10 180 python -u $R/tools/infer_case.py $sc | grep res=
    done
  done
done
