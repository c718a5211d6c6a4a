# round-6 GPU check: the GPU test suite, then the module-path child (timing +
# rocprofv3 breakdown), each step under its own time limit
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06}
mkdir -p $O
F="--no-cpu-baseline --no-kernel-timing --no-alt-backward --no-shading --no-infer --no-traffic --no-c5 --no-module-path"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 240 python bench.py --eager --module-path-child --steps 20 --warmup 10 $F > $O/module_eager.log 2>&1 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_module -o run -- python $R/bench.py --eager --module-path-child --steps 20 --warmup 10 $F > $O/prof_module.log 2>&1
