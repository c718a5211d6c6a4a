#!/bin/bash
# Walk bound probe: the binned backward per walk mode with the slice-image adds
# as built (0), on bank-distinct rows (1) and removed (2) — variant libraries
# lib/libdfhip_probe{1,2}.so built beforehand (tools/variant_lib.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-probe}
mkdir -p $OUT
for p in 0 1 2; do
  if [ $p = 0 ]; then unset DFHIP_LIB; else export DFHIP_LIB=$PWD/single-stable-dreamfusion_amd/lib/libdfhip_probe$p.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p$p -o run \
      -- python tools/grid_bin_case.py --modes ${MODES:-0,3,1} --ranges 0-15 --reps 5 > $OUT/p$p.log 2>&1 \
      || { echo "probe $p failed"; tail -20 $OUT/p$p.log; exit 3; }
  echo "=== probe $p"; grep median $OUT/p$p.log
  python tools/prof_top.py $OUT/p$p/run_kernel_stats.csv 6
done
