# fold-binning probe A/B: the fused forward walked tile-owner by tile-owner
# (lib/libdfhip_foldprobe.so, tools/fold_probe.py) against the product
# library, same bench child, interleaved twice
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06d}
mkdir -p $O
F="--no-cpu-baseline --no-kernel-timing --no-alt-backward --no-shading --no-infer --no-traffic --no-c5 --no-module-path"
cd /tmp
for rep in 1 2; do
  for v in base foldprobe; do
    if [ $v = base ]; then unset DFHIP_LIB; else export DFHIP_LIB=$R/single-stable-dreamfusion_amd/lib/libdfhip_$v.so; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v$rep -o run -- python $R/bench.py --steps 30 --warmup 10 $F > $O/$v$rep.log 2>&1 || exit 1
    echo "== $v rep $rep"; python $R/tools/prof_top.py $O/$v$rep/run_kernel_stats.csv 6
  done
done
