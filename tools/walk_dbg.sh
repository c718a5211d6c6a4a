#!/bin/bash
# k_walk experiment switches (DFHIP_WALK_DBG, csrc/gridbin.hip BinInfo::dbg):
# rocprofv3 kernel stats of the binned grid backward of a real march per switch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for d in ${DBGS:-0 1 2 3 4}; do
    out=gpurun_out/wd/d$d
    mkdir -p $out
    DFHIP_WALK_DBG=$d timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $out -o run -- python3 tools/grid_bin_case.py --reps 5 --ranges ${RANGES:-0-15} \
        > $out/log 2>&1 || { echo "dbg $d failed"; tail -5 $out/log; exit 1; }
    echo "dbg=$d"
    python3 tools/prof_top.py $(find $out -name "*kernel_stats.csv" | head -1) 4
done
