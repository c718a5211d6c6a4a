# C4 march: the occupied path's next byte prefetched one step ahead
# (-DDFHIP_RENDER_PREFETCH=1 build as lib/libdfhip_pf.so; the option was
# removed after this A/B) vs without: render tests with it, then infer_case
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
L=$R/single-stable-dreamfusion_amd/lib
DFHIP_LIB=$L/libdfhip_pf.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_render.py > gpurun_out/r06ad_test.txt 2>&1
tail -1 gpurun_out/r06ad_test.txt
for sc in "" "--sphere"; do
  for i in 1 2 3; do
    for v in base pf; do
      if [ $v = base ]; then unset DFHIP_LIB; else export DFHIP_LIB=$L/libdfhip_$v.so; fi
      echo "== $v $sc"; timeout -k 10 180 python -u $R/tools/infer_case.py $sc | grep res=
    done
  done
done
