# kept-clean binned scratch A/B (DFHIP_KEPT_CLEAN=0: the per-step fill launch)
# interleaved three times, to separate its effect from the run-to-run spread
# of k_walk seen in r06f / r06g (183 vs 217 us by run)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06h}
mkdir -p $O
F="--no-cpu-baseline --no-kernel-timing --no-alt-backward --no-shading --no-infer --no-traffic --no-c5 --no-module-path"
timeout -k 10 300 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_native_step.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
cd /tmp
for rep in 1 2 3; do
  for v in 1 0; do
    export DFHIP_KEPT_CLEAN=$v
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kc$v.$rep -o run -- python $R/bench.py --steps 30 --warmup 10 $F > $O/kc$v.$rep.log 2>&1 || exit 1
    echo "== kept_clean=$v rep $rep $(grep -o '"ms_per_step": [0-9.]*' $O/kc$v.$rep.log | head -1)"; python $R/tools/prof_top.py $O/kc$v.$rep/run_kernel_stats.csv 30 | grep -E "k_walkIDF|fillBuffer|total"
  done
done
