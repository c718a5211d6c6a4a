# Train march count: ray groups dispatched centre-out (a -DDFHIP_MARCH_CENTER=1 build,
# since removed) vs in ray order; rocprofv3 of the C2 child, alternating
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06r}
mkdir -p $O
F="--steps 40 --warmup 10 --no-cpu-baseline --no-kernel-timing --no-alt-backward --no-shading --no-infer --no-traffic --no-c5 --no-module-path"
cd /tmp
for rep in 1 2; do
  for v in base center; do
    if [ $v = center ]; then export DFHIP_LIB=$R/single-stable-dreamfusion_amd/lib/libdfhip_center.so; else unset DFHIP_LIB; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v$rep -o run -- python $R/bench.py $F > $O/$v$rep.log 2>&1 || exit 1
    echo "== $v $rep $(grep -o '"ms_per_step": [0-9.]*' $O/$v$rep.log | head -1)"; python $R/tools/prof_top.py $O/$v$rep/run_kernel_stats.csv 30 | grep -E "march_train|total"
  done
done
