# albedo native step without per-sample dirs in the emit: tests, then the C2
# child under rocprofv3 twice
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06o}
mkdir -p $O
F="--no-cpu-baseline --no-kernel-timing --no-alt-backward --no-shading --no-infer --no-traffic --no-c5 --no-module-path"
timeout -k 10 600 python -u -m pytest tests/test_gpu_native_step.py tests/test_gpu_raymarching.py tests/test_gpu_shading.py tests/test_gpu_step_structures.py tests/test_gpu_graph.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
cd /tmp
for rep in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$rep -o run -- python $R/bench.py --steps 30 --warmup 10 $F > $O/p$rep.log 2>&1 || exit 1
  echo "== rep $rep $(grep -o '"ms_per_step": [0-9.]*' $O/p$rep.log | head -1)"; python $R/tools/prof_top.py $O/p$rep/run_kernel_stats.csv 30 | grep -E "march_train|k_walkIDF|total"
done
