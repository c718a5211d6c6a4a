# module path after the tile-gather grid forward: encoder / module tests, the
# module child timed, its host profile and its rocprofv3 breakdown; then the
# C4 hand-off A/B
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06b}
mkdir -p $O
F="--no-cpu-baseline --no-kernel-timing --no-alt-backward --no-shading --no-infer --no-traffic --no-c5 --no-module-path"
timeout -k 10 400 python -u -m pytest tests/test_gpu_encoders.py tests/test_gpu_module_path.py tests/test_gpu_render.py -m gpu -x -v --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 240 python bench.py --eager --module-path-child --steps 20 --warmup 10 $F > $O/module_eager.log 2>&1 &&
timeout -k 10 240 python tools/host_profile.py 60 --module > $O/host_module.log 2>&1 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_module -o run -- python $R/bench.py --eager --module-path-child --steps 20 --warmup 10 $F > $O/prof_module.log 2>&1 &&
cd $R && timeout -k 10 400 python tools/infer_handoff_ab.py --values 0,8,16,24,32 --reps 10 --rounds 2 > $O/handoff_ab.log 2>&1
