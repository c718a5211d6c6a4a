# one-launch GradScaler + Adam and the kept-clean binned scratch in the
# replayed step: their tests, then an A/B of the C2 bench child (=0: the three
# Adam launches and the scratch fill), interleaved twice; then the module leg
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06f}
mkdir -p $O
F="--no-cpu-baseline --no-kernel-timing --no-alt-backward --no-shading --no-infer --no-traffic --no-c5 --no-module-path"
timeout -k 10 600 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_native_step.py tests/test_gpu_graph.py tests/test_gpu_rccl.py tests/test_gpu_bf16.py tests/test_gpu_module_path.py tests/test_gpu_encoders.py -m gpu -x -v --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
cd /tmp
for rep in 1 2; do
  for v in 1 0; do
    export DFHIP_FUSED_ADAM=$v DFHIP_KEPT_CLEAN=$v
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/adam$v.$rep -o run -- python $R/bench.py --steps 30 --warmup 10 $F > $O/adam$v.$rep.log 2>&1 || exit 1
    echo "== fused=$v rep $rep"; python $R/tools/prof_top.py $O/adam$v.$rep/run_kernel_stats.csv 25
  done
done
unset DFHIP_FUSED_ADAM DFHIP_KEPT_CLEAN
cd $R
timeout -k 10 600 python -c "
import sys, json; sys.argv=['bench.py','--steps','20','--warmup','10']; sys.path[:0]=['.','single-stable-dreamfusion_amd']
import bench; a=bench.parse(); print(json.dumps(bench.module_path_leg(a)))" > $O/module_leg.log 2>&1
