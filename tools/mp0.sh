# module-path variants (reference-API modules, autograd body) on one box
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/mp0
F="--no-cpu-baseline --no-kernel-timing --no-alt-backward --no-shading --no-infer --no-traffic --no-c5 --no-module-path"
export DFHIP_NATIVE_STEP=0 DFHIP_FUSED_FIELD=0
timeout -k 10 240 python bench.py --steps 20 --warmup 10 $F > $R/gpurun_out/mp0/graph_cap.log 2>&1 &&
timeout -k 10 240 python bench.py --eager --steps 20 --warmup 10 $F > $R/gpurun_out/mp0/eager_sliced.log 2>&1 &&
DFHIP_GRID_BWD=atomic timeout -k 10 240 python bench.py --eager --steps 20 --warmup 10 $F > $R/gpurun_out/mp0/eager_atomic.log 2>&1 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/mp0/prof -o run -- python $R/bench.py --eager --steps 20 --warmup 10 $F > $R/gpurun_out/mp0/prof.log 2>&1
