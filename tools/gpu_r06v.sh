# C4 eval frame: the background net on a side stream beside the fused render
# (renderer.infer_overlap_bg) vs after it: render tests, infer_case A/B
# interleaved, and one rocprofv3 kernel trace of each (the overlap in time)
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06v
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_render.py > $O/test.txt 2>&1
tail -1 $O/test.txt
for sc in "" "--sphere"; do
  for i in 1 2 3; do
    for v in "" "--serial-bg"; do
      echo "== ${v:-overlap} $sc"; timeout -k 10 180 python -u $R/tools/infer_case.py $sc $v | grep res=
    done
  done
done
cd /tmp
for v in "" "--serial-bg"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr${v:-_overlap} -o run -- python $R/tools/infer_case.py --reps 5 $v > $O/tr${v:-_overlap}.log 2>&1
done
