# module path as bucketed graphs: its tests, the module leg of bench.py
# (graph child, eager child, rocprofv3 breakdown), and the render tests
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06c}
mkdir -p $O
F="--no-cpu-baseline --no-kernel-timing --no-alt-backward --no-shading --no-infer --no-traffic --no-c5 --no-module-path"
timeout -k 10 400 python -u -m pytest tests/test_gpu_module_path.py tests/test_gpu_render.py tests/test_gpu_graph.py -m gpu -x -v --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py --module-path-child --steps 20 --warmup 10 $F > $O/module_graph.log 2>&1 &&
timeout -k 10 600 python -c "
import sys, json; sys.argv=['bench.py','--steps','20','--warmup','10']; sys.path[:0]=['.','single-stable-dreamfusion_amd']
import bench; a=bench.parse(); print(json.dumps(bench.module_path_leg(a)))" > $O/module_leg.log 2>&1
