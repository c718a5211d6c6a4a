# C4 march: the empty-cell skip loop with the constant dt of dt_gamma = 0
# (-DDFHIP_MARCH_G0=1 build as lib/libdfhip_g0.so) vs the general loop:
# render tests with it, then infer_case (the option was removed after this A/B)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
L=$R/single-stable-dreamfusion_amd/lib
DFHIP_LIB=$L/libdfhip_g0.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_render.py > gpurun_out/r06ae_test.txt 2>&1
tail -1 gpurun_out/r06ae_test.txt
for sc in "" "--sphere"; do
  for i in 1 2 3; do
    for v in base g0; do
      if [ $v = base ]; then unset DFHIP_LIB; else export DFHIP_LIB=$L/libdfhip_$v.so; fi
      echo "== $v $sc"; timeout -k 10 180 python -u $R/tools/infer_case.py $sc | grep res=
    done
  done
done
