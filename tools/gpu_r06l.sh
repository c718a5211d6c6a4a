# walk plan longest-part-first (default) vs bin order (DFHIP_PLAN_LPT=0): its
# tests, then the C2 bench child and the textureless child under rocprofv3,
# interleaved twice
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06l}
mkdir -p $O
F="--no-cpu-baseline --no-kernel-timing --no-alt-backward --no-shading --no-infer --no-traffic --no-c5 --no-module-path"
timeout -k 10 600 python -u -m pytest tests/test_gpu_encoders.py tests/test_gpu_native_step.py tests/test_gpu_module_path.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
cd /tmp
for rep in 1 2; do
  for v in 1 0; do
    export DFHIP_PLAN_LPT=$v
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lpt$v.$rep -o run -- python $R/bench.py --steps 30 --warmup 10 $F > $O/lpt$v.$rep.log 2>&1 || exit 1
    echo "== plan_lpt=$v rep $rep $(grep -o '"ms_per_step": [0-9.]*' $O/lpt$v.$rep.log | head -1)"; python $R/tools/prof_top.py $O/lpt$v.$rep/run_kernel_stats.csv 30 | grep -E "k_walk|k_sum2|total"
  done
done
for v in 1 0; do
  export DFHIP_PLAN_LPT=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tx$v -o run -- python $R/bench.py --shade textureless --steps 30 --warmup 10 $F > $O/tx$v.log 2>&1 || exit 1
  echo "== textureless plan_lpt=$v $(grep -o '"ms_per_step": [0-9.]*' $O/tx$v.log | head -1)"; python $R/tools/prof_top.py $O/tx$v/run_kernel_stats.csv 30 | grep -E "k_walk|k_sum2|total"
done
