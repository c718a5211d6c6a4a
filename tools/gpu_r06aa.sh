# C4 march: the empty-cell skip loop in closed form (-DDFHIP_SKIP_BITS=1 build
# as lib/libdfhip_sb.so; the option was removed after this A/B) vs the loop:
# render tests with it, then infer_case R0 / R1 interleaved
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
L=$R/single-stable-dreamfusion_amd/lib
DFHIP_LIB=$L/libdfhip_sb.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_render.py > gpurun_out/r06aa_test.txt 2>&1
tail -1 gpurun_out/r06aa_test.txt
for sc in "" "--sphere"; do
  for i in 1 2 3; do
    for v in base sb; do
      if [ $v = base ]; then unset DFHIP_LIB; else export DFHIP_LIB=$L/libdfhip_$v.so; fi
      echo "== $v $sc"; timeout -k 10 180 python -u $R/tools/infer_case.py $sc | grep res=
    done
  done
done
