#!/bin/bash
# Kernel stats of the windowed vs slice backward on one level range ($1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
r=${1:-0-0}
for mode in win slices; do
    out=gpurun_out/gbab/$mode$r
    mkdir -p $out
    if [ $mode = slices ]; then export DFHIP_GRID_NOWIN=1; fi
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run \
        -- python3 tools/grid_bin_case.py --reps 5 --ranges $r > $out/log 2>&1 || { echo "failed"; tail -5 $out/log; exit 1; }
    echo "== $mode $r: $(grep median $out/log)"
    python3 tools/prof_top.py $(find $out -name "*kernel_stats.csv" | head -1) 4
done
