# ray head forward + backward as one launch in the native step: its tests,
# then an A/B of the C2 bench child (DFHIP_COMBINED_HEAD=0: two launches),
# interleaved twice
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06i}
mkdir -p $O
F="--no-cpu-baseline --no-kernel-timing --no-alt-backward --no-shading --no-infer --no-traffic --no-c5 --no-module-path"
timeout -k 10 600 python -u -m pytest tests/test_gpu_native_step.py tests/test_gpu_network.py tests/test_gpu_field_oracle.py tests/test_gpu_step_structures.py tests/test_gpu_bf16.py tests/test_gpu_shading.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
cd /tmp
for rep in 1 2; do
  for v in 1 0; do
    export DFHIP_COMBINED_HEAD=$v
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ch$v.$rep -o run -- python $R/bench.py --steps 30 --warmup 10 $F > $O/ch$v.$rep.log 2>&1 || exit 1
    echo "== combined_head=$v rep $rep $(grep -o '"ms_per_step": [0-9.]*' $O/ch$v.$rep.log | head -1)"; python $R/tools/prof_top.py $O/ch$v.$rep/run_kernel_stats.csv 30 | grep -E "hd::|k_walkIDF|total"
  done
done
