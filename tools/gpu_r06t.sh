# Final round-6 check: the GPU suite, smoke(), the
# default bench, and the C4 leg under rocprofv3 (tiles vs row strips)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06t}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 600 python -u $R/bench.py > $O/bench.log 2>&1 || exit 1
grep '^{' $O/bench.log | tail -1 > $O/bench.json
F="--no-cpu-baseline --no-kernel-timing --no-alt-backward --no-shading --no-traffic --no-c5 --no-module-path"
cd /tmp
for v in 1 0; do
  DFHIP_INFER_TILES=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4_t$v -o run -- python $R/bench.py --steps 10 --warmup 5 $F > $O/c4_t$v.log 2>&1 || exit 1
  echo "== tiles $v"; python $R/tools/prof_top.py $O/c4_t$v/run_kernel_stats.csv 40 | grep -E "render_infer|chunk|total"
done
