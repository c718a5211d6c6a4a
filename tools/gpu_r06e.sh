# stencil-walk gather probe (tools/walk_gather_probe.py): the product library
# against gradlocal (gradient rows from L1-resident slots, same control flow)
# and alllocal (positions too), textureless child twice interleaved, then the
# albedo child once
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06e}
mkdir -p $O
F="--no-cpu-baseline --no-kernel-timing --no-alt-backward --no-shading --no-infer --no-traffic --no-c5 --no-module-path"
cd /tmp
run() {  # variant shade tag
  if [ $1 = base ]; then unset DFHIP_LIB; else export DFHIP_LIB=$R/single-stable-dreamfusion_amd/lib/libdfhip_$1.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$1_$3 -o run -- python $R/bench.py --shade $2 --steps 30 --warmup 10 $F > $O/$1_$3.log 2>&1 || exit 1
  echo "== $1 $3"; python $R/tools/prof_top.py $O/$1_$3/run_kernel_stats.csv 6
}
for rep in 1 2; do
  for v in base gradlocal alllocal; do run $v textureless tx$rep; done
done
for v in base gradlocal alllocal; do run $v albedo alb; done
cd $R
unset DFHIP_LIB
timeout -k 10 600 python -c "
import sys, json; sys.argv=['bench.py','--steps','20','--warmup','10']; sys.path[:0]=['.','single-stable-dreamfusion_amd']
import bench; a=bench.parse(); print(json.dumps(bench.module_path_leg(a)))" > $O/module_leg.log 2>&1
