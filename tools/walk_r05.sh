#!/bin/bash
# Round-5 walk study: per-workgroup timelines of the per-segment walk (mode 0)
# and the resolved stream (mode 3), then SQ counters of both walks and bins,
# then the binning A/B against lib/libdfhip_${VAR:-ballot4}.so.
# Record of round 5 only: walk mode 3 and the binning variants it drives were
# removed from the library in round 6.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-walk_r05}
mkdir -p $OUT
for m in 0 3; do
  timeout -k 10 200 python -u tools/walk_trace.py --mode $m --reps 3 > $OUT/trace$m.log 2>&1 \
      || { echo "trace $m failed"; tail -20 $OUT/trace$m.log; exit 1; }
  echo "=== timeline mode $m"; head -12 $OUT/trace$m.log
done
for m in 0 3; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_BUSY_CYCLES \
      --output-format csv -d $OUT/pmc$m -o p1 -- python3 tools/grid_bin_case.py --modes $m --ranges 0-15 --reps 3 > $OUT/pmc$m.log 2>&1 \
      || { echo "pmc $m failed"; tail -5 $OUT/pmc$m.log; exit 2; }
  echo "=== counters mode $m"
  for k in k_walk k_rwalk k_rbin k_bin_fast; do python3 tools/pmc_table.py $OUT/pmc$m $k; done
done
VAR=${VAR:-ballot4} TAG=${TAG:-walk_r05}_binab bash tools/bin_ab.sh
# the stencil walk with the slice-image adds on bank-distinct rows (probe 1)
# and removed (probe 2): their share of k_walk_flat<7>
for p in 1 2; do
  export DFHIP_LIB=$PWD/single-stable-dreamfusion_amd/lib/libdfhip_probe$p.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/shprobe$p -o run \
      -- python tools/shade_steps.py textureless 20 > $OUT/shprobe$p.log 2>&1 \
      || { echo "shade probe $p failed"; tail -20 $OUT/shprobe$p.log; exit 5; }
  echo "=== textureless probe $p"; python tools/prof_top.py $OUT/shprobe$p/run_kernel_stats.csv 4
done
